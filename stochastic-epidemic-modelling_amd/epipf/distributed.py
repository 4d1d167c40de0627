"""Multi-GPU PMCMC: independent chains sharded one process per GPU, one gather at the end.

SURVEY.md §8e: the reference's independent chains are separate runs later combined by Gelman-Rubin
(tests/test_pmcmc_p.py:303-308, helpers.py:15-43).  Here rank r of a `torch.distributed` job (backend
"nccl" = RCCL over xGMI on MI355X; "gloo" on CPU for tests) runs its contiguous shard of the global chain
ids with no collective on the data path (`scaling: weak`).  The only exchange is `gather_draws`: one
all-gather of every chain's posterior draws (theta, log-likelihood), after which every rank holds all
chains in global-chain order and computes their Gelman-Rubin R-hat (helpers.py:15-43).  Each rank can also
write its chains in the reference's CSV layout and resume them from a warm start.  Chain g uses host RandomState(seed + g) and Philox key chain_key(seed, g)
on whichever rank runs it, so a run's draws do not depend on the number of GPUs.
"""
import os
from typing import NamedTuple, Optional

import numpy as np

from .chains_io import gelman_rubin, load_run, save_run, warm_start


def shard(total_chains, world, rank):
    """Global chain ids of `rank`: contiguous blocks, the first `total % world` ranks get one more."""
    base, extra = divmod(int(total_chains), int(world))
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def _tensor_device(dist, device):
    return f"cuda:{device}" if dist.get_backend() == "nccl" else "cpu"


def gather_draws(draws, device=0, force=False):
    """All-gather a per-rank float64 array [C_local, ...] (C_local may differ by one between ranks) into
    [C_total, ...] on every rank, in rank order.  Without an initialised process group, returns `draws`; with a
    one-rank group the collective still runs when `force` is set (exercises RCCL init and device tensors)."""
    import torch
    import torch.distributed as dist
    draws = np.ascontiguousarray(draws, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return draws
    if dist.get_world_size() == 1 and not force:
        return draws
    dev = _tensor_device(dist, device)
    world = dist.get_world_size()
    n = torch.tensor([draws.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    cmax = max(counts)
    pad = np.zeros((cmax,) + draws.shape[1:], dtype=np.float64)
    pad[:draws.shape[0]] = draws
    t = torch.from_numpy(pad).to(dev)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return np.concatenate([o.cpu().numpy()[:c] for o, c in zip(out, counts)], axis=0)


def pack_draws(results, upto=None):
    """[C, iters*d + iters] rows of (thetas flattened, log-likelihoods) from ChainResult objects."""
    if not results:
        return np.stack([])                                   # numpy's own error for no chains, as before
    n = len(results[0].log_likelihoods) if upto is None else min(int(upto), len(results[0].log_likelihoods))
    d = results[0].thetas.shape[1]
    out = np.empty((len(results), n * d + n))
    th_out, ll_out = out[:, :n * d].reshape(-1, n, d), out[:, n * d:]
    for k, r in enumerate(results):                           # one row per chain, written in place
        th_out[k] = r.thetas[:n]
        ll_out[k] = r.log_likelihoods[:n]
    return out


def unpack_draws(packed, d):
    """Inverse of pack_draws: (thetas [C, iters, d], log_likelihoods [C, iters])."""
    iters = packed.shape[1] // (d + 1)
    return packed[:, :iters * d].reshape(-1, iters, d), packed[:, iters * d:]


class ShardedRun(NamedTuple):
    """Result of sharded_pmcmc: this rank's ChainResults and global chain ids, every chain's gathered draws
    (thetas [total, iters, d], log-likelihoods [total, iters]) and the Gelman-Rubin R-hat per parameter of the
    gathered chains after `burn_in` (helpers.py:15-43; None with fewer than two chains)."""
    results: list
    ids: list
    thetas: np.ndarray
    log_likelihoods: np.ndarray
    rhat: Optional[np.ndarray]


def chain_dir(directory, g):
    """Per-chain run directory of a sharded run (one reference-layout run per chain, chains_io.save_run)."""
    return os.path.join(directory, f"chain_{int(g):04d}")


def resume_points(directory, ids, burn_in=100, thin=20):
    """Warm starts of chains `ids` from their saved runs (tests/test_pmcmc_noisy.py:32-40 per chain):
    (parameters [n, d], sigma [n, d, d])."""
    starts = [warm_start(load_run(chain_dir(directory, g))[0], burn_in, thin) for g in ids]
    return np.array([s[0] for s in starts]), np.stack([s[1] for s in starts])


def sharded_pmcmc(Y, type_model, parameters, h, total_chains, *, seed=0, device=0, burn_in=0, save_dir=None,
                  resume_dir=None, resume_burn_in=100, resume_thin=20, force_gather=False, **kw):
    """Run `total_chains` independent PMCMC chains over the ranks of the current process group (or all on this
    process when none is initialised) and all-gather their draws (one collective, at the end).

    save_dir: each rank writes its chains in the reference's layout (tests/experiments/pobs/prob_.05.py:57-61),
    one directory per global chain id (chain_dir).  resume_dir: every chain starts from the warm start of its own
    saved run there (last draw, covariance of the burned-in thinned unique draws; `sigma` is then per chain).
    The gathered thetas give R-hat over all chains after `burn_in` iterations (every rank computes the same value).
    Returns a ShardedRun."""
    from .pmcmc import chain_key, particle_mcmc_chains
    try:
        import torch.distributed as dist
        on = dist.is_available() and dist.is_initialized()
    except ImportError:  # pragma: no cover
        on = False
    world = dist.get_world_size() if on else 1
    rank = dist.get_rank() if on else 0
    ids = shard(total_chains, world, rank)
    rngs = [np.random.RandomState(seed + g) for g in ids]
    keys = [chain_key(seed, g) for g in ids]
    d = np.asarray(parameters).shape[-1]
    if resume_dir is not None and ids:
        parameters, kw["sigma"] = resume_points(resume_dir, ids, resume_burn_in, resume_thin)
    res = particle_mcmc_chains(Y, type_model, parameters, h, rngs=rngs, keys=keys, device=device, **kw) if ids else []
    if save_dir is not None:
        for g, r in zip(ids, res):
            save_run(chain_dir(save_dir, g), r.thetas, r.likelihoods, r.sampled_trajs)
    packed = pack_draws(res) if res else np.zeros((0, kw.get("n_chains", 1000) * (d + 1)))
    allp = gather_draws(packed, device, force=force_gather)
    th, ll = unpack_draws(allp, d)
    rhat = gelman_rubin(list(th[:, burn_in:])) if th.shape[0] >= 2 and th.shape[1] - burn_in >= 2 else None
    return ShardedRun(res, ids, th, ll, rhat)
