"""Multi-GPU PMCMC: independent chains sharded one process per GPU, one gather at the end.

SURVEY.md §8e: the reference's independent chains are separate runs later combined by Gelman-Rubin
(tests/test_pmcmc_p.py:303-308, helpers.py:15-43).  Here rank r of a `torch.distributed` job (backend
"nccl" = RCCL over xGMI on MI355X; "gloo" on CPU for tests) runs its contiguous shard of the global chain
ids with no collective on the data path (`scaling: weak`).  The only exchange is `gather_draws`: one
all-gather of every chain's posterior draws (theta, log-likelihood), after which every rank holds all
chains in global-chain order.  Chain g uses host RandomState(seed + g) and Philox key chain_key(seed, g)
on whichever rank runs it, so a run's draws do not depend on the number of GPUs.
"""
import numpy as np


def shard(total_chains, world, rank):
    """Global chain ids of `rank`: contiguous blocks, the first `total % world` ranks get one more."""
    base, extra = divmod(int(total_chains), int(world))
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def _tensor_device(dist, device):
    return f"cuda:{device}" if dist.get_backend() == "nccl" else "cpu"


def gather_draws(draws, device=0):
    """All-gather a per-rank float64 array [C_local, ...] (C_local may differ by one between ranks) into
    [C_total, ...] on every rank, in rank order.  Without an initialised process group, returns `draws`."""
    import torch
    import torch.distributed as dist
    draws = np.ascontiguousarray(draws, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
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
    rows = []
    for r in results:
        th = r.thetas if upto is None else r.thetas[:upto]
        ll = r.log_likelihoods if upto is None else r.log_likelihoods[:upto]
        rows.append(np.concatenate([th.reshape(-1), ll]))
    return np.stack(rows)


def unpack_draws(packed, d):
    """Inverse of pack_draws: (thetas [C, iters, d], log_likelihoods [C, iters])."""
    iters = packed.shape[1] // (d + 1)
    return packed[:, :iters * d].reshape(-1, iters, d), packed[:, iters * d:]


def sharded_pmcmc(Y, type_model, parameters, h, total_chains, *, seed=0, device=0, **kw):
    """Run `total_chains` independent PMCMC chains over the ranks of the current process group (or all
    on this process when none is initialised).  Returns (local ChainResults, local chain ids, gathered
    thetas [total, iters, d], gathered log-likelihoods [total, iters])."""
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
    res = particle_mcmc_chains(Y, type_model, parameters, h, rngs=rngs, keys=keys, device=device, **kw) if ids else []
    d = len(parameters)
    packed = pack_draws(res) if res else np.zeros((0, kw.get("n_chains", 1000) * (d + 1)))
    allp = gather_draws(packed, device)
    th, ll = unpack_draws(allp, d)
    return res, ids, th, ll
