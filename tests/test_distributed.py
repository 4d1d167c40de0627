"""Multi-process chain sharding on CPU: world_size-2 `gloo` jobs run their shards of the
global chains and all-gather the draws; the gathered posterior must equal a one-process run of every
chain.  The filter is the oracle test double (tests/oracle_engine.py); on MI355X the same code runs with
backend "nccl" (RCCL) and the HIP engine (bench.py --gpus N)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from epipf import distributed as D
from epipf import pmcmc as pm
from oracle_engine import fake_get_engine

HERE = os.path.dirname(os.path.abspath(__file__))

KW = dict(adaptive=False, sigma=None, n_chains=5, observations=False, probs=0.1, n_particles=12, n_population=200,
          mu=20, mh_ratio="log")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, Y, total, paths, q, prefetch=0):
    for p in paths:
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from epipf import distributed as Dw
    from epipf import pmcmc as pmw
    from oracle_engine import fake_get_engine as fge
    pmw.get_engine = fge
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res, ids, th, ll = Dw.sharded_pmcmc(Y, "sir", [2.0, 1.0], 0.01, total, seed=9, prefetch=prefetch, **KW)
        q.put((rank, ids, th, ll))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_shard_partitions_chains():
    for total in range(0, 11):
        for world in (1, 2, 3, 8):
            ids = [D.shard(total, world, r) for r in range(world)]
            flat = [g for s in ids for g in s]
            assert flat == list(range(total))
            assert max(map(len, ids)) - min(map(len, ids)) <= 1


def test_pack_unpack_roundtrip():
    class R:
        pass
    rs = np.random.RandomState(0)
    res = []
    for _ in range(3):
        r = R()
        r.thetas, r.log_likelihoods = rs.rand(7, 2), rs.rand(7)
        res.append(r)
    th, ll = D.unpack_draws(D.pack_draws(res), 2)
    for c in range(3):
        np.testing.assert_array_equal(th[c], res[c].thetas)
        np.testing.assert_array_equal(ll[c], res[c].log_likelihoods)


@pytest.mark.parametrize("total,prefetch", [(3, 0), (4, 0), (2, 4)])
def test_gloo_world2_gather_equals_single_process(monkeypatch, datasets_golden, total, prefetch):
    """prefetch > 0 with one chain per rank is the north star's one-chain-per-GPU layout, each chain speculative;
    the gathered draws equal a one-process lockstep run of every chain."""
    Y = datasets_golden["cfg1_binom"][:6]
    monkeypatch.setattr(pm, "get_engine", fake_get_engine)
    _, ids, th1, ll1 = D.sharded_pmcmc(Y, "sir", [2.0, 1.0], 0.01, total, seed=9, **KW)
    assert ids == list(range(total))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    paths = [HERE] + [p for p in sys.path if "stochastic-epidemic" in p or p.endswith("oracle")]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, Y, total, paths, q, prefetch)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, ids_r, th, ll = q.get(timeout=240)
        out[rank] = (ids_r, th, ll)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][0] + out[1][0] == list(range(total))
    for rank in (0, 1):
        np.testing.assert_array_equal(out[rank][1], th1)   # every rank holds all chains, in global order
        np.testing.assert_array_equal(out[rank][2], ll1)
