"""Where one MH iteration's wall time goes for a small batch (default: BASELINE config 5, one chain): the whole
ChainSampler.step(), the filter call alone (Engine.run), the path-sampler call alone (Engine.path_sample), and the
device time of the filter's kernels (HIP events, PROFILE_TIMING).  The differences are host work and round trips.
  python scripts/mh_iteration_probe.py [--cfg 5] [--chains 1] [--iters 200]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
from epipf import _lib, datasets  # noqa: E402
from epipf.pmcmc import ChainSampler, chain_key  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", type=int, default=5)
ap.add_argument("--chains", type=int, default=1)
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--h", type=float, default=1e-4)
ap.add_argument("--tag", default="")
ap.add_argument("--particles", type=int, default=0, help="override the config's N")
args = ap.parse_args()

Y, meta = datasets.benchmark_dataset(args.cfg)
N, T = (args.particles or meta["N"]), Y.shape[0]
nc = args.chains
s = ChainSampler(Y, meta["model"], list(meta["theta"]), args.h, sigma=meta["sigma"], iters=2 * args.iters + 10,
                 observations=meta.get("observations", False), probs=meta["probs"], n_particles=N,
                 n_population=meta["n_population"], mu=meta["mu"],
                 rngs=[np.random.RandomState(7 + c) for c in range(nc)], keys=[chain_key(7, c) for c in range(nc)],
                 mh_ratio="log")
s.initialise()
for _ in range(5):
    s.step()


def per_call(fn, n):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6, float(np.mean(ts)) * 1e6


step_med, step_mean = per_call(s.step, args.iters)
eng = s.eng
th = np.tile(np.asarray(s.thetas[0, s.i - 1][:s.dth]), (nc, 1))
fi = [10 ** 6]


def run():
    fi[0] += 1
    eng.run(th, s.probs if s.probs is not None else 0.1, s.keys, np.full(nc, fi[0], dtype=np.uint64),
            observations=s.observations)


run_med, run_mean = per_call(run, args.iters)
chosen = np.zeros(nc, dtype=np.int32)
ps_med, ps_mean = per_call(lambda: eng.path_sample(chosen), args.iters)
eng.reset_stats()
eng.set_profiling(_lib.PROFILE_TIMING)
for _ in range(args.iters):
    run()
st = eng.stats()
eng.set_profiling(_lib.PROFILE_OFF)
dev_us = (st["init_ms"] + st["step_ms"]) / args.iters * 1e3
out = dict(tag=args.tag, fused=int(st.get("last_fused", 0)), cfg=args.cfg, chains=nc, N=N, T=T, h=args.h, lanes=int(st.get("last_lanes", 0)),
           step_us_median=step_med, step_us_mean=step_mean, run_us_median=run_med, run_us_mean=run_mean,
           path_sample_us_median=ps_med, device_filter_us_mean=dev_us,
           host_and_round_trips_us=step_mean - dev_us,
           particle_steps_per_s_step=nc * N * T / (step_mean * 1e-6))
print(json.dumps(out), flush=True)
