"""Filter throughput vs SSA lanes per particle (epipf_set_lanes) and chains per launch, BASELINE configs 2 and 5.

    python scripts/lanes_sweep.py [--cfg 2 5] [--chains 1 2 4 8 16] [--lanes 1 2 4 8 16] [--reps 3]

One JSON line per (config, chains, lanes): particle-steps/s of whole filters (epipf_run wall time, host included),
median over reps, plus the automatic choice's lanes for that chain count."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, nargs="+", default=[2, 5])
    ap.add_argument("--chains", type=int, nargs="+", default=[1, 2, 4, 8, 16])
    ap.add_argument("--lanes", nargs="+", default=["1", "4", "8", "16"],
                    help="W or W:K (lanes per particle : events per lane per chunk; K 0 = automatic)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--particles", type=int, nargs="+", default=[0],
                    help="particles per chain (0 = the config's N); per-particle work does not depend on N")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "lanes_sweep.jsonl"))
    args = ap.parse_args()
    from epipf import datasets
    from epipf.engine import model_id, theta_vector
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "a") as fo:
        for cfg in args.cfg:
            Y, meta = datasets.benchmark_dataset(cfg)
            mid = model_id(meta["model"])
            base = np.asarray(meta["theta"], dtype=np.float64)
            G = int(round(np.sqrt(base.size - 1))) if mid >= 2 else 1
            th = theta_vector(mid, (base[:G * G].reshape(G, G), base[-1]) if mid >= 2 else tuple(base))[0]
            for N in args.particles:
                sweep(args, fo, cfg, Y, meta, mid, G, th, N or meta["N"])


def sweep(args, fo, cfg, Y, meta, mid, G, th, N):
    from epipf.engine import Engine
    T = Y.shape[0]
    eng = Engine(meta["model"], G, N, T, max(args.chains))
    eng.set_observations(Y)
    eng.set_population(meta["n_population"], meta["mu"])
    obs = bool(meta.get("observations", False))
    f = 0
    for chains in args.chains:
        eng.set_lanes(0, 0)
        eng.run(np.tile(th, (chains, 1)), [meta["probs"]] * chains, list(range(1, chains + 1)), [f] * chains,
                observations=obs)
        auto = eng.stats()["last_lanes"]
        for spec in args.lanes:
            lanes, _, kk = spec.partition(":")
            lanes, kk = int(lanes), int(kk or 0)
            eng.set_lanes(lanes, kk)
            ts = []
            for r in range(args.reps + 1):
                f += 1
                t0 = time.perf_counter()
                eng.run(np.tile(th, (chains, 1)), [meta["probs"]] * chains, list(range(1, chains + 1)),
                        [f] * chains, observations=obs)
                if r:
                    ts.append(time.perf_counter() - t0)
            dt = float(np.median(ts))
            rec = dict(cfg=cfg, chains=chains, lanes=lanes, lane_events=eng.stats()["last_lane_events"],
                       auto_lanes=auto, N=N, T=T,
                       ms_per_filter_batch=dt * 1e3, particle_steps_per_s=N * T * chains / dt)
            print(json.dumps(rec), flush=True)
            fo.write(json.dumps(rec) + "\n")
    eng.close()


if __name__ == "__main__":
    main()
