"""Diagnostic: torch's HIP runtime after libepipf's has initialised the device (and the environment around it)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
env0 = dict(os.environ)
import numpy as np  # noqa: E402
from epipf.engine import Engine  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "torch-first":
    import torch
    print("torch first: device_count", torch.cuda.device_count(), flush=True)
eng = Engine("sir", 1, 100, 5, 1)
eng.set_observations(np.zeros((5, 3)))
eng.set_population(200, 20)
eng.run(np.array([[2.0, 1.0]]), [0.1], [1], [0])
print("epipf ran; env changes:", {k: v for k, v in os.environ.items() if env0.get(k) != v}, flush=True)
import torch  # noqa: E402
print("torch.cuda.device_count()", torch.cuda.device_count(), flush=True)
try:
    torch.cuda.set_device(0)
    print("set_device ok", torch.zeros(3, device="cuda").sum().item(), flush=True)
except Exception as e:  # noqa: BLE001
    print("set_device failed:", e, flush=True)
eng.close()
