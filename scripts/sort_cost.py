"""Cost of the per-step sort an ordering-by-predicted-work scheme needs: sort each
chain's N = 10^4 particle keys (predicted work, with the particle index as value) for 256 chains, every filter step,
on the GPU (torch.sort along dim 1 = rocPRIM segmented radix sort).  Compared with the modelled gain of ordering:
lane use 0.830 -> 0.855 (scripts/lane_use_model.py) on a ~470 us step launch per chain group."""
import json
import time

import torch


def main():
    dev = torch.device("cuda:0")
    out = {}
    for chains in (64, 256):
        keys = torch.randint(0, 1 << 16, (chains, 10000), device=dev, dtype=torch.int32)
        for _ in range(3):
            torch.sort(keys, dim=1)
        torch.cuda.synchronize()
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            v, idx = torch.sort(keys, dim=1)
        torch.cuda.synchronize()
        out[f"sort_us_{chains}_chains"] = (time.perf_counter() - t0) / reps * 1e6
    # what ordering could buy per step of 256 chains: the SSA share of a step x the lane-use gain
    step_us = 4 * 470.0 / 4 * 4 / 4 * 1.0            # one step of all 256 chains ~ 470 us wall (4 concurrent groups)
    out["step_wall_us_256_chains"] = step_us
    out["modelled_gain_us"] = step_us * 0.91 * (1 - 0.830 / 0.855)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
