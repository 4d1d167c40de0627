"""ABC rejection throughput on MI355X (abc_algo.py:17-109), one JSON line.

Workload: the reference's own ABC setting, tests/test_abc_sir.py:43 -- abc_algo(sir_noisy (T=15), 1000
samples, threshold 150, priors beta, gamma ~ U[0, 5]).  value = trials/s of whole epipf_abc runs (batched
rejection loop, select + gather included); also the kernel-only trial rate (HIP events), SSA events/s, SIMD
lane use (device counters, separate run) and the CPU oracle (OpenMP C restatement) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1000)
    ap.add_argument("--threshold", type=float, default=150.0)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    from epipf import _lib
    from epipf.engine import get_engine
    Y = np.load(os.path.join(REPO, "tests", "golden", "datasets.npz"))["sir_noisy"]
    pr = {"beta": [0.0, 5.0], "gamma": [0.0, 5.0]}
    eng = get_engine("sir", 1, 1, 1, 1)
    eng.abc(Y, args.samples, args.threshold, pr, 1, 999, batch=args.batch)         # warm-up
    eng.set_profiling(_lib.PROFILE_TIMING)
    eng.reset_stats()
    t0 = time.perf_counter()
    trials = 0
    for r in range(args.runs):
        _, _, tr, acc = eng.abc(Y, args.samples, args.threshold, pr, 2024, r, batch=args.batch)
        assert acc == args.samples
        trials += tr
    wall = time.perf_counter() - t0
    st = eng.stats()
    simulated = st["abc_trials"]
    eng.set_profiling(_lib.PROFILE_COUNTERS)
    eng.reset_stats()
    eng.abc(Y, args.samples, args.threshold, pr, 2024, 0, batch=args.batch)
    sc = eng.stats()
    eng.set_profiling(_lib.PROFILE_OFF)

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    oracle.build()
    t1 = time.perf_counter()
    n_cpu = 0
    while time.perf_counter() - t1 < args.cpu_seconds:
        oracle.abc_trials(Y, pr, 2024, 0, n_cpu, 2000, rows=False)
        n_cpu += 2000
    cpu_dt = time.perf_counter() - t1
    line = {
        "metric": "abc_trials_per_second", "value": trials / wall, "unit": "trials/s", "higher_is_better": True,
        "workload": "abc_algo(sir_noisy T=15, n=%d, threshold=%g, U[0,5]^2 priors) -- tests/test_abc_sir.py:43"
                    % (args.samples, args.threshold),
        "runs": args.runs, "reference_trials_per_run": trials / args.runs, "wall_s": wall,
        "samples_per_s": args.samples * args.runs / wall,
        "trials_simulated_incl_batch_overshoot": simulated,
        "kernel_trials_per_s": simulated / (st["abc_ms"] / 1e3) if st["abc_ms"] else None,
        "kernel_ms": st["abc_ms"], "launches": st["abc_launches"],
        "events_per_trial": sc["events"] / max(sc["abc_trials"], 1),
        "events_per_s_kernel": sc["events"] / max(sc["abc_trials"], 1) * simulated / (st["abc_ms"] / 1e3)
        if st["abc_ms"] else None,
        "lane_use": sc["lane_iterations"] / sc["wave_lane_slots"] if sc["wave_lane_slots"] else None,
        "cpu_baseline": {"value": n_cpu / cpu_dt, "unit": "trials/s", "cores": oracle.num_threads(), "kind": "port",
                         "sample": f"{n_cpu} trials of the same run (oracle/abc_oracle.c), {cpu_dt:.1f}s"},
    }
    line["gpu_over_cpu"] = line["value"] / line["cpu_baseline"]["value"]
    print(json.dumps(line))


if __name__ == "__main__":
    main()
