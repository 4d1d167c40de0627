"""The C-ABI library loads and exports every entry point include/epipf.h declares (CPU-safe: no
compute calls, no device needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "epipf.h")
LIB = os.path.join(PKG, "lib", "libepipf.so")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(epipf_[a-z_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("epipf_create", "epipf_run", "epipf_path_sample", "epipf_simulate", "epipf_resample"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    L = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_python_binding_lists_every_symbol():
    from epipf import _lib
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_abi_version_and_device_query():
    from epipf import _lib
    L = _lib.load()
    assert L.epipf_abi_version() == _lib.ABI_VERSION
    assert L.epipf_device_count() >= 0


def test_create_without_device_fails_loudly():
    """No CPU fallback: on a GPU-less host the engine refuses to construct."""
    from epipf import _lib
    from epipf.engine import Engine
    if _lib.load().epipf_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.EpipfError):
        Engine("sir", 1, 16, 4, 1)


def test_constants_match_header():
    from epipf import _lib
    text = open(HEADER).read()
    defs = dict(re.findall(r"#define (EPIPF_\w+) \(?(-?\d+)\)?", text))
    assert int(defs["EPIPF_STATUS_DEGENERATE"]) == _lib.STATUS_DEGENERATE
    assert int(defs["EPIPF_SIR_SUBGROUPS2"]) == _lib.SIR_SUBGROUPS2
    assert int(defs["EPIPF_RESAMPLE_SYSTEMATIC"]) == _lib.RESAMPLE_SYSTEMATIC
    assert int(defs["EPIPF_ABI_VERSION"]) == _lib.ABI_VERSION
    assert int(defs["EPIPF_PROFILE_TIMING"]) == _lib.PROFILE_TIMING
    assert int(defs["EPIPF_PROFILE_COUNTERS"]) == _lib.PROFILE_COUNTERS


def makefile_build_id():
    """The id csrc/Makefile stamps into the libraries: sha256 of the exact source, header, script and Makefile list
    it names (csrc/Makefile BUILD_ID), evaluated by make itself."""
    out = subprocess.run(["make", "-s", "--no-print-directory", "-C", os.path.join(PKG, "csrc"), "build-id"],
                         check=True, capture_output=True, text=True).stdout.strip()
    assert len(out) == 16 and int(out, 16) >= 0, out
    return out


def test_build_id_matches_the_sources():
    """The loaded libepipf.so was built from the sources in this tree: a stale prebuilt library (pushed to the GPU box
    next to edited sources) fails here, and with it every PMC profile bench.py would match on its id."""
    from epipf import _lib
    assert _lib.build_id() == makefile_build_id(), "libepipf.so is stale: rebuild (__graft_entry__.build())"


def test_debug_library_exports_the_same_boundary():
    """libepipf_debug.so (make debug: device traps, roctx ranges) is a drop-in for libepipf.so."""
    path = os.path.join(PKG, "lib", "libepipf_debug.so")
    assert os.path.exists(path), "run __graft_entry__.build() first"
    D = ctypes.CDLL(path)
    assert not [s for s in declared_symbols() if not hasattr(D, s)]
    D.epipf_build_id.restype = ctypes.c_char_p
    from epipf import _lib
    assert D.epipf_build_id().decode() == makefile_build_id() + "-debug", "libepipf_debug.so is stale"


@pytest.mark.gpu
def test_build_ids_match_the_sources_where_the_library_runs():
    """The same two checks in the GPU run (the CPU-only check never ran on the box that receives the
    prebuilt libraries): libepipf.so and libepipf_debug.so carry the build id of the sources shipped beside them."""
    test_build_id_matches_the_sources()
    test_debug_library_exports_the_same_boundary()
