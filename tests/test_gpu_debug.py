"""The debug library (libepipf_debug.so: `make -C stochastic-epidemic-modelling_amd/csrc debug`) -- device traps in
place of the release build's index clamps, roctx ranges per filter call and step -- runs the 96-case randomised
parity sweep (tests/test_gpu_fuzz.py) green: no ancestor or path index ever leaves [0, N).  One child process with
EPIPF_LIBRARY pointing at the debug library (the binding reads it at import)."""
import os
import subprocess
import sys

import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

DRIVER = r"""
import sys
sys.path[:0] = [{tests!r}, {pkg!r}, {oracle!r}, {repo!r}]
from epipf import _lib
assert _lib.LIB_PATH.endswith("libepipf_debug.so"), _lib.LIB_PATH
assert _lib.build_id().endswith("-debug"), _lib.build_id()
import test_gpu_fuzz as f
n = 0
for seed in range(96):
    f.test_random_filters_match_oracle(seed)
    n += 1
print("debug fuzz cases green:", n, "build", _lib.build_id(), flush=True)
"""


def test_debug_library_runs_the_fuzz_sweep():
    lib = os.path.join(PKG, "lib", "libepipf_debug.so")
    assert os.path.exists(lib), "build() makes libepipf_debug.so"
    code = DRIVER.format(tests=os.path.join(REPO, "tests"), pkg=PKG, oracle=os.path.join(REPO, "oracle"), repo=REPO)
    env = dict(os.environ, EPIPF_LIBRARY=lib)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "debug fuzz cases green: 96" in r.stdout
