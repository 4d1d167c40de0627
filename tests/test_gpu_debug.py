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
    if not os.path.exists(lib):
        pytest.skip("no libepipf_debug.so: build() makes it where the roctx SDK is present")
    code = DRIVER.format(tests=os.path.join(REPO, "tests"), pkg=PKG, oracle=os.path.join(REPO, "oracle"), repo=REPO)
    env = dict(os.environ, EPIPF_LIBRARY=lib)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "debug fuzz cases green: 96" in r.stdout


DRIVER_STATUS = r"""
import sys
sys.path[:0] = [{pkg!r}, {repo!r}]
import numpy as np
from epipf import _lib
from epipf.engine import Engine
assert _lib.LIB_PATH.endswith("libepipf_debug.so"), _lib.LIB_PATH
z = np.load({golden!r})
Y = z["sir_binom"][:8]
eng = Engine("sir", 1, 300, Y.shape[0], 3)
eng.set_observations(Y)
eng.set_population(4820, 20)
# chain 0 ordinary; chain 1 degenerate (p = 1e-300: every binomial weight underflows to 0); chain 2 skipped
lz, st = eng.run(np.array([[2.0, 1.0]] * 3), [0.1, 1e-300, 0.1], [1, 2, 3], [0, 0, 0], active=np.array([1, 1, 0]))
assert st[0] == _lib.STATUS_OK and st[1] == _lib.STATUS_DEGENERATE and st[2] == _lib.STATUS_SKIPPED, st
tr = eng.path_sample(np.array([7, 7, 7], dtype=np.int32))
assert tr[0].sum() > 0 and not tr[1].any() and not tr[2].any()
hid, anc = eng.history(1)
np.testing.assert_array_equal(tr[0][-1], hid[0][-1, 7])
print("path sampler skipped the non-OK chains without a trap", flush=True)
"""


def test_debug_library_path_sampler_skips_failed_chains():
    """The path sampler walks only chains whose last run was OK: a degenerate chain's and a skipped chain's history
    rows may be stale or unwritten (the step kernels return early once a chain fails), and the debug library traps on
    any ancestor index outside [0, N) -- so walking them could trap a normal call.  ADVICE r3."""
    lib = os.path.join(PKG, "lib", "libepipf_debug.so")
    if not os.path.exists(lib):
        pytest.skip("no libepipf_debug.so: build() makes it where the roctx SDK is present")
    code = DRIVER_STATUS.format(pkg=PKG, repo=REPO, golden=os.path.join(REPO, "tests", "golden", "datasets.npz"))
    env = dict(os.environ, EPIPF_LIBRARY=lib)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "skipped the non-OK chains" in r.stdout
