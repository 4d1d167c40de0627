"""Host-side paths on the device: the RCCL all-gather of a sharded run (backend "nccl" = RCCL on ROCm, one rank),
Gelman-Rubin and CSV output of the gathered chains, and samplers that share one cached engine.  `-m gpu`."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_world1_gather_rhat_and_csv(datasets_golden, tmp_path):
    """sharded_pmcmc over a one-rank RCCL group with the all-gather forced: RCCL init, device tensors and the
    collective run; gathered draws equal the local chains, R-hat equals helpers.py:15-43 restated on them, and each
    chain's CSVs are byte-identical to np.savetxt of its results (tests/experiments/pobs/prob_.05.py:57-61)."""
    import torch
    import torch.distributed as dist
    from epipf import distributed as D
    from epipf.chains_io import gelman_rubin, save_run
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        Y = datasets_golden["sir_binom"]
        run = D.sharded_pmcmc(Y, "sir", [2.0, 1.0], 0.05, 4, seed=3, device=0, n_chains=12, n_particles=300,
                              n_population=4820, mu=20, probs=0.1, mh_ratio="log", save_dir=str(tmp_path / "run"),
                              burn_in=2, force_gather=True)
    finally:
        dist.destroy_process_group()
    assert run.ids == [0, 1, 2, 3]
    for c, r in enumerate(run.results):
        np.testing.assert_array_equal(run.thetas[c], r.thetas)
        np.testing.assert_array_equal(run.log_likelihoods[c], r.log_likelihoods)
        ref = tmp_path / f"ref{c}"
        save_run(str(ref), r.thetas, r.likelihoods, r.sampled_trajs)
        for f in sorted(os.listdir(ref)):
            assert (ref / f).read_bytes() == open(os.path.join(D.chain_dir(str(tmp_path / "run"), c), f), "rb").read()
    np.testing.assert_array_equal(run.rhat, gelman_rubin([r.thetas[2:] for r in run.results]))
    assert run.rhat.shape == (2,) and np.all(np.isfinite(run.rhat))


def test_samplers_sharing_a_cached_engine_keep_their_data(datasets_golden):
    """Two lockstep samplers with different observations and populations but the same model / N share one cached
    engine; interleaving their steps gives each exactly the draws it gets when run alone."""
    from epipf import pmcmc as pm
    from epipf.engine import _CACHE
    Ya = datasets_golden["sir_binom"]
    Yb = np.floor(0.9 * Ya)            # other binomial counts of the same shape (never all-zero weights)

    def sampler(Y, npop, seed):
        return pm.ChainSampler(Y, "sir", [2.0, 1.0], 0.05, iters=6, probs=0.1, n_particles=256, n_population=npop,
                               mu=20, rngs=[np.random.RandomState(seed)], keys=[pm.chain_key(seed, 0)], mh_ratio="log")

    alone = []
    for Y, npop, seed in ((Ya, 4820, 1), (Yb, 5000, 2)):
        _CACHE.clear()
        s = sampler(Y, npop, seed)
        s.run()
        alone.append(s.results()[0])
    _CACHE.clear()
    a, b = sampler(Ya, 4820, 1), sampler(Yb, 5000, 2)
    assert a.eng is b.eng
    a.initialise()
    b.initialise()
    for _ in range(5):
        a.step()
        b.step()
    for s, ref in ((a, alone[0]), (b, alone[1])):
        r = s.results()[0]
        np.testing.assert_array_equal(r.thetas, ref.thetas)
        np.testing.assert_array_equal(r.log_likelihoods, ref.log_likelihoods)
        np.testing.assert_array_equal(r.sampled_trajs, ref.sampled_trajs)


def test_engine_growth_keeps_live_sampler_working(datasets_golden):
    """A particle_filter call that needs a larger horizon replaces the cached engine; a sampler still holding the
    old one keeps running on it (it is released with its last reference, not closed under the sampler)."""
    from epipf import pmcmc as pm
    from epipf.engine import _CACHE
    _CACHE.clear()
    Y = datasets_golden["sir_binom"]
    s = pm.ChainSampler(Y, "sir", [2.0, 1.0], 0.05, iters=4, probs=0.1, n_particles=128, n_population=4820, mu=20,
                        rngs=[np.random.RandomState(5)], keys=[pm.chain_key(5, 0)], mh_ratio="log")
    s.initialise()
    old = s.eng
    Y2 = datasets_golden["cfg1_binom"]                    # 50 rows > 15: a bigger context replaces the cached one
    z, _, _ = pm.particle_filter(Y2, "sir", (2.0, 1.0), n_particles=128, n_population=200, key=3, filter_index=0)
    assert z is not None
    from epipf.engine import model_id
    assert _CACHE[(model_id("sir"), 1, 128, 0)] is not old
    s.step()
    s.step()
    assert s.i == 3
