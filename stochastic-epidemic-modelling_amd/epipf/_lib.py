"""ctypes binding of libepipf.so (the C ABI declared in include/epipf.h).

The library is the product: there is no CPU fallback.  If it is missing or the device is absent,
every entry point raises immediately.
"""
import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("EPIPF_LIBRARY", os.path.join(PKG_ROOT, "lib", "libepipf.so"))

# constants mirrored from include/epipf.h
OK, EINVAL, EHIP, ENOMEM, ESTATE = 0, -1, -2, -3, -4
STATUS_OK, STATUS_DEGENERATE, STATUS_SKIPPED = 0, 1, 2
SIR, SEIR, SIR_SUBGROUPS, SIR_SUBGROUPS2 = 0, 1, 2, 3
OBS_BINOMIAL, OBS_NORMAL = 0, 1
RESAMPLE_MULTINOMIAL, RESAMPLE_SYSTEMATIC = 0, 1
PROFILE_OFF, PROFILE_TIMING, PROFILE_COUNTERS = 0, 1, 2
ABI_VERSION = 8

EXPORTS = (
    "epipf_create", "epipf_destroy", "epipf_set_observations", "epipf_set_population", "epipf_run",
    "epipf_run_sampled", "epipf_mh_propose", "epipf_mh_decide", "epipf_mh_peek",
    "epipf_copy_history", "epipf_path_sample", "epipf_simulate", "epipf_resample", "epipf_set_profiling",
    "epipf_get_stats", "epipf_reset_stats", "epipf_set_streams", "epipf_set_lanes", "epipf_last_error", "epipf_abi_version", "epipf_device_count",
    "epipf_build_id",
    "epipf_abc", "epipf_abc_trials", "epipf_glibc_log", "epipf_clock_log", "epipf_simulate_path",
)


class Stats(ctypes.Structure):
    _fields_ = [
        ("step_ms", ctypes.c_double),
        ("step_launches", ctypes.c_int64),
        ("init_ms", ctypes.c_double),
        ("init_launches", ctypes.c_int64),
        ("events", ctypes.c_int64),
        ("particle_steps", ctypes.c_int64),
        ("filters", ctypes.c_int64),
        ("resample_fallbacks", ctypes.c_int64),
        ("lane_iterations", ctypes.c_int64),
        ("wave_lane_slots", ctypes.c_int64),
        ("abc_ms", ctypes.c_double),
        ("abc_launches", ctypes.c_int64),
        ("abc_trials", ctypes.c_int64),
        ("ssa_exact_lanes", ctypes.c_int64),
        ("ssa_exact_waves", ctypes.c_int64),
        ("step_kernel_ms", ctypes.c_double),
        ("step_kernel_launches", ctypes.c_int64),
        ("last_lanes", ctypes.c_int64),
        ("last_lane_events", ctypes.c_int64),
        ("resample_ref_ambiguous", ctypes.c_int64),
        ("last_fused", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class EpipfError(RuntimeError):
    pass


_lib = None


def load():
    """Load libepipf.so once; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EpipfError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                         "(the HIP path has no CPU fallback)")
    # One HIP runtime per process: torch (device memory, streams, RCCL for the multi-GPU gather) ships its own
    # libamdhip64 / ROCr.  Loaded first, the library's HIP dependency resolves to that same runtime; loaded after
    # libepipf's, torch's second runtime finds no GPU ("No HIP GPUs are available", scripts/torch_after_epipf.py).
    # EPIPF_NO_TORCH_PRELOAD=1 skips it for callers that never touch torch.  A torch that fails to import for any reason
    # (a ROCm library mismatch raises OSError / RuntimeError, not ImportError) leaves the library loadable on its own.
    if os.environ.get("EPIPF_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except Exception:  # noqa: BLE001
            pass
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    i32, u32, u64, f64 = ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double
    sig = {
        "epipf_create": ([ctypes.POINTER(P), i32, i32, i32, i32, i32, i32], i32),
        "epipf_destroy": ([P], None),
        "epipf_set_observations": ([P, P, i32, i32], i32),
        "epipf_set_population": ([P, P, P], i32),
        "epipf_run": ([P, i32, P, i32, i32, P, P, P, P, i32, P, P], i32),
        "epipf_run_sampled": ([P, i32, P, i32, i32, P, P, P, P, i32, P, P, P, P], i32),
        "epipf_mh_propose": ([i32, i32, P, P, P, P, P], i32),
        "epipf_mh_decide": ([i32, P, P, i32, P, P, P, P], i32),
        "epipf_mh_peek": ([i32, P, P, i32, P], i32),
        "epipf_copy_history": ([P, i32, P, P], i32),
        "epipf_path_sample": ([P, i32, P, P], i32),
        "epipf_simulate": ([P, i32, P, P, i32, f64, u64, u32, u32, P, P], i32),
        "epipf_resample": ([P, i32, P, P, P, P], i32),
        "epipf_set_profiling": ([P, i32], i32),
        "epipf_set_streams": ([P, i32], i32),
        "epipf_set_lanes": ([P, i32, i32], i32),
        "epipf_get_stats": ([P, ctypes.POINTER(Stats)], i32),
        "epipf_reset_stats": ([P], i32),
        "epipf_last_error": ([], ctypes.c_char_p),
        "epipf_abi_version": ([], i32),
        "epipf_build_id": ([], ctypes.c_char_p),
        "epipf_device_count": ([], i32),
        "epipf_abc": ([P, P, i32, i32, f64, P, u64, u32, ctypes.c_int64, i32, P, P, P, P], i32),
        "epipf_abc_trials": ([P, P, i32, P, u64, u32, u32, i32, P, P, P, P], i32),
        "epipf_glibc_log": ([ctypes.c_int64, P, P], i32),
        "epipf_clock_log": ([ctypes.c_int64, P, P], i32),
        "epipf_simulate_path": ([P, i32, P, P, i32, f64, u64, u32, u32, i32, P, P, P, P], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.epipf_abi_version() != ABI_VERSION:
        raise EpipfError(f"libepipf.so ABI {L.epipf_abi_version()} != expected {ABI_VERSION}")
    _lib = L
    return L


def build_id():
    """The loaded library's build id (epipf_build_id: hash of its sources and flags)."""
    return load().epipf_build_id().decode()


def check(rc, what):
    if rc < 0:
        msg = load().epipf_last_error().decode(errors="replace")
        raise EpipfError(f"{what} failed ({rc}): {msg}")
    return rc


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None
