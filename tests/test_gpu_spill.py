"""The lane-group kernel under a forced low register budget (libepipf_spill.so: `make -C
stochastic-epidemic-modelling_amd/csrc spill`, every pf_step_group_kernel instance built with EPIPF_GROUP_MIN_WAVES=8,
i.e. 64 VGPRs and heavy scratch spills) is bit-exact to the oracle: spilling must not change results (a
rejected round-5 variant with 29 spills returned wrong states).  One child process with EPIPF_LIBRARY
pointing at the spill library runs the lane-group parity cases of tests/test_gpu_lanes.py -- every model and width,
G = 3 and 4, the widened decision band (the exact-fallback redo), the exact-clock redo -- and BASELINE configs 5
and 2 at full size on one chain (W = 16) against the oracle (/root/reference/gillespie_algo.py:148-233)."""
import os
import subprocess
import sys

import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

DRIVER = r"""
import sys, os
sys.path[:0] = [{tests!r}, {pkg!r}, {oracle!r}, {repo!r}]
import numpy as np
from epipf import _lib
assert _lib.LIB_PATH.endswith("libepipf_spill.so"), _lib.LIB_PATH
assert _lib.build_id().endswith("-spill"), _lib.build_id()
import conftest
import test_gpu_lanes as t
dg = {{k: v for k, v in np.load(os.path.join({golden!r}, "datasets.npz")).items()}}


class MP:                                    # monkeypatch.setenv for the child (engines read the variables at create)
    def setenv(self, k, v):
        os.environ[k] = v


n = 0
for model in ["sir", "sir_normal", "seir", "sir_subgroups", "sir_subgroups2"]:
    for lanes in [2, 4, 8, 16]:
        t.test_lane_groups_match_oracle(dg, model, lanes)
        n += 1
for G in (3, 4):
    t.test_lane_groups_larger_subgroup_models_equal_one_lane(dg, G)
    n += 1
for model in ["sir", "seir", "sir_subgroups"]:
    for lanes in (8, 16):
        os.environ.pop("EPIPF_CLOCK_SLACK", None)
        t.test_certified_clock_redo_equals_oracle(dg, MP(), model, lanes)
        os.environ.pop("EPIPF_CLOCK_SLACK", None)
        n += 1
for model in ["sir", "sir_subgroups", "sir_subgroups2"]:
    t.test_widened_decision_band_equals_oracle(dg, MP(), model, 8)
    os.environ.pop("EPIPF_BAND_SLACK", None)
    n += 1
for cfg in (5, 2):
    t.test_lane_groups_full_size_single_chain_vs_oracle(cfg, 0)
    n += 1
print("spill-build lane-group cases green:", n, "build", _lib.build_id(), flush=True)
"""


def test_forced_spill_build_is_bit_exact_to_the_oracle():
    lib = os.path.join(PKG, "lib", "libepipf_spill.so")
    if not os.path.exists(lib):
        pytest.skip("no libepipf_spill.so: __graft_entry__.build() makes it")
    code = DRIVER.format(tests=os.path.join(REPO, "tests"), pkg=PKG, oracle=os.path.join(REPO, "oracle"), repo=REPO,
                         golden=os.path.join(REPO, "tests", "golden"))
    env = {k: v for k, v in os.environ.items() if not k.startswith("EPIPF_")}
    env["EPIPF_LIBRARY"] = lib
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "spill-build lane-group cases green: 33" in r.stdout, r.stdout[-2000:]
