"""Build-time self-check of the device log's table (make runs it after linking libepipf.so; a mismatch deletes the
library and fails the build).  gen_glibc_log.py copies glibc's __log_data table out of this machine's libm and
glibc_log_impl (epipf_device.hpp) restates the FMA variant of glibc's log around it; if the host's libm differed
(another glibc version, the non-FMA path, another table layout) the restatement would silently stop being the
reference's math.log.  epipf_glibc_log runs that exact code on the CPU: compare it with libm's log (math.log) on
2*10^5 inputs -- the SSA's 1 - U range, values next to 1 (the table-free path), and a wide range of magnitudes.
Usage: python3 check_glibc_log.py <libepipf.so>"""
import ctypes
import math
import sys

import numpy as np


def main(path):
    L = ctypes.CDLL(path)
    L.epipf_glibc_log.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    L.epipf_glibc_log.restype = ctypes.c_int
    rs = np.random.RandomState(20240)
    x = np.concatenate([
        1.0 - (rs.randint(0, 2**53, 100000, dtype=np.int64) >> 0).astype(np.float64) * 2.0**-53,   # 1 - U
        1.0 + rs.uniform(-0.07, 0.07, 40000),                                                     # near 1
        np.exp(rs.uniform(-700, 700, 40000)),                                                     # wide range
        rs.uniform(2.0**-53, 2.0**-20, 20000),                                                    # tiny 1 - U
    ])
    x = x[(x > 0) & np.isfinite(x)]
    out = np.empty_like(x)
    rc = L.epipf_glibc_log(x.size, x.ctypes.data, out.ctypes.data)
    if rc != 0:
        sys.exit(f"epipf_glibc_log returned {rc}")
    want = np.array([math.log(v) for v in x.tolist()])
    bad = np.nonzero(out.view(np.int64) != want.view(np.int64))[0]
    if bad.size:
        i = int(bad[0])
        sys.exit(f"device log restatement differs from this host's libm log on {bad.size} of {x.size} inputs "
                 f"(first: log({x[i]!r}) = {want[i]!r}, restatement {out[i]!r}): the copied table or the glibc "
                 f"variant does not match -- the library must not be used")
    print(f"glibc log self-check: {x.size} inputs bit-identical to libm")


if __name__ == "__main__":
    main(sys.argv[1])
