"""Ancestors against the reference itself, at bench scale, in the driver's GPU suite.

The device's binomial weight is the true pmf to an ulp; the reference's is scipy's binom.pmf (pmcmc.py:179), which is
itself off by up to ~1e-12 relative.  So the device's ancestors equal the reference's wherever scipy's
own error cannot move a CDF boundary across a draw -- which the device counts as `resample_ref_ambiguous`.  These
tests run the bench's filters on the GPU (config 2: 66 chains x N = 10^4 x T = 200 = 1.31e8 resampling draws, the
one-lane kernel of the bench; configs 3 and 5 at full size, the lane-group kernel) and replay every step of every chain
the reference's way on the host: scipy.stats weights of the device's own states (pmcmc.py:177-181), numpy's legacy
choice on the keyed uniforms (:185-190; tests/reference_replay.py).  0 ancestors may differ; the ambiguity count is
printed beside it.  Host replay in a spawn pool (subprocesses, no exec of this GPU process)."""
import json
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _replay(job):
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "oracle")]
    import reference_replay
    Y, hid, anc, model, obs, probs, key, f = job
    return reference_replay.replay(Y, hid, anc, model, obs, probs, key, f)


@pytest.mark.parametrize("cfg,chains,lanes,slice_", [(2, 66, 1, 22), (3, 16, 0, 8), (5, 64, 0, 8)])
def test_reference_replay_at_bench_scale(cfg, chains, lanes, slice_):
    from epipf import _lib, datasets
    from epipf.engine import Engine
    from epipf.pmcmc import chain_key
    Y, meta = datasets.benchmark_dataset(cfg)
    G = len(np.atleast_1d(meta["n_population"]))
    th = np.asarray(meta["theta"], dtype=np.float64)
    N, T = meta["N"], Y.shape[0]
    obs = bool(meta.get("observations", False))
    rs = np.random.RandomState(2024 + cfg)
    thetas = np.abs(th[None] * (1.0 + 0.05 * rs.standard_normal((chains, th.size))))   # around the bench's start
    keys = [chain_key(2024, g) for g in range(chains)]
    eng = Engine(meta["model"], G, N, T, slice_)
    eng.set_observations(Y)
    eng.set_population(meta["n_population"], meta["mu"])
    eng.set_lanes(lanes)
    eng.set_profiling(_lib.PROFILE_COUNTERS)
    draws = bad = n_ok = 0
    ctx = mp.get_context("spawn")
    with ctx.Pool(min(16, max(2, (os.cpu_count() or 4) // 2))) as pool:
        for lo in range(0, chains, slice_):
            n = min(slice_, chains - lo)
            lz, st = eng.run(thetas[lo:lo + n], [meta["probs"]] * n, keys[lo:lo + n], [3] * n, observations=obs)
            if lanes == 0:                                # <= 8 chains of 10^4: the lane-group kernel
                assert eng.stats()["last_lanes"] > 1
            hid, anc = eng.history(n)
            jobs = [(Y, hid[c], anc[c], meta["model"], obs, meta["probs"], keys[lo + c], 3) for c in range(n)
                    if st[c] == 0]
            n_ok += len(jobs)
            del hid, anc
            for d, b in pool.map(_replay, jobs):
                draws += d
                bad += b
    stats = eng.stats()
    eng.close()
    rec = {"config": cfg, "chains": chains, "chains_ok": n_ok, "draws_replayed": draws,
           "ancestors_differing_from_reference": bad, "device_resample_ref_ambiguous": stats["resample_ref_ambiguous"],
           "device_uncertified_draws": stats["resample_fallbacks"], "lanes": stats["last_lanes"],
           "library_build_id": _lib.build_id()}
    print(f"config {cfg}: {draws} resampling draws of {n_ok} chains replayed the reference's way, {bad} ancestors "
          f"differ; device reference-ambiguous draws {stats['resample_ref_ambiguous']}, uncertified "
          f"{stats['resample_fallbacks']}, lanes {stats['last_lanes']}")
    out = os.path.join(os.path.dirname(HERE), "gpurun_out")             # the record, beside the test log
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"ref_replay_cfg{cfg}.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    assert n_ok >= chains - 1
    if cfg == 2:
        assert draws >= 1.3e8
    assert bad == 0
