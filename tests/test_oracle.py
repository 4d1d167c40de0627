"""Pin the CPU oracle (oracle/) before trusting it: Philox known-answer vectors, and every golden
fixture produced by running the unmodified reference (tests/golden/make_golden.py)."""
import numpy as np
import pytest

import oracle
import philox as ph
from conftest import case_args

# Random123 kat_vectors for philox4x32-10 (Salmon et al., SC'11)
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,expected", KAT)
def test_philox_kat_numpy(ctr, key, expected):
    out = ph.philox4x32_10(*ctr, key)
    assert tuple(int(x) for x in out) == expected


@pytest.mark.parametrize("ctr,key,expected", KAT)
def test_philox_kat_c(ctr, key, expected):
    out = oracle.philox(*ctr, key[0] | (key[1] << 32))
    assert tuple(int(x) for x in out) == expected


def test_philox_c_matches_numpy_stream():
    rs = np.random.RandomState(0)
    for _ in range(200):
        c = rs.randint(0, 2**32, 4, dtype=np.uint64)
        key = int(rs.randint(0, 2**63, dtype=np.int64)) * 2 + 1
        a = oracle.philox(*[int(x) for x in c], key)
        b = ph.philox4x32_10(*c, ph.split_key(key))
        assert [int(x) for x in a] == [int(x) for x in b]


FILTER_CASES = ["sir_binom", "sir_normal", "seir_binom", "sub_binom", "sub2_binom", "cfg1_sir", "cfg2_sir",
                "cfg3_seir_normal", "sir_theta_off", "degenerate"]


@pytest.mark.parametrize("name", FILTER_CASES)
def test_oracle_filter_matches_reference(filter_golden, name):
    """Integer outputs bit-exact, zetas within 1e-9 relative (scipy's Boost pmf vs lgamma restatement)."""
    rec = filter_golden["filter_" + name]
    a = case_args(rec)
    o = oracle.particle_filter(a["Y"], a["model"], a["theta"], a["observations"], a["probs"], a["N"], a["npop"],
                               a["mu"], key=a["key"], filter_index=a["f"])
    assert o["status"] == int(rec["status"])
    if o["status"]:
        return
    np.testing.assert_array_equal(o["hidden"], rec["hidden"])
    np.testing.assert_array_equal(o["ancestry"], rec["ancestry"])
    z = rec["zetas"]
    finite = z > 1e-290  # the reference's linear product loses precision once subnormal
    np.testing.assert_allclose(o["zetas"][finite], z[finite], rtol=1e-9, atol=0)
    # log-space likelihood agrees wherever the reference's linear product has not underflowed
    np.testing.assert_allclose(o["log_zetas"][finite], np.log(z[finite]), rtol=0, atol=1e-9)


@pytest.mark.parametrize("name", ["sir_1.0", "sir_2.5", "sir_edge_1.0", "sir_edge_2.5", "seir_1.0", "seir_2.5",
                                  "sub_1.0", "sub_2.5"])
def test_oracle_ssa_matches_reference(kernels_golden, name):
    rec = kernels_golden["ssa_" + name]
    model = str(rec["model"])
    theta = (rec["theta"][:4].reshape(2, 2), float(rec["theta"][4])) if model == "sub" else rec["theta"]
    mname = {"sir": "sir", "seir": "seir", "sub": "sir_subgroups"}[model]
    out, _ = oracle.simulate(mname, rec["states"], theta, float(rec["max_time"]), int(rec["key"]), int(rec["f"]),
                             int(rec["step"]))
    np.testing.assert_array_equal(out, rec["out"])


@pytest.mark.parametrize("n", [1, 2, 5, 64, 257, 1000])
def test_oracle_resample_matches_numpy_choice(kernels_golden, n):
    rec = kernels_golden[f"resample_{n}"]
    np.testing.assert_array_equal(oracle.resample(rec["w"], rec["u"]), rec["expected"])


def test_oracle_resample_degenerate():
    assert oracle.resample(np.zeros(8), np.full(8, 0.5)) is None
    w = np.ones(8)
    w[3] = np.nan
    assert oracle.resample(w, np.full(8, 0.5)) is None


def test_oracle_binom_pmf_matches_scipy(kernels_golden):
    rec = kernels_golden["pmf_binom"]
    got = oracle.binom_pmf(rec["k"], rec["n"], rec["p"])
    exp = rec["pmf"]
    np.testing.assert_array_equal(got == 0, exp == 0)
    nz = exp > 1e-300
    np.testing.assert_allclose(got[nz], exp[nz], rtol=1e-9)


def test_oracle_norm_pdf_matches_scipy(kernels_golden):
    rec = kernels_golden["pdf_normal"]
    got = oracle.norm_pdf(rec["y"], rec["x"], rec["probs"])
    np.testing.assert_allclose(got, rec["pdf"], rtol=1e-14, atol=0)


def test_poisson_inversion_numpy_matches_c():
    """The golden shim's initial draws (numpy inversion) equal the oracle's (C) on the same stream."""
    Y = np.ones((2, 3))
    o = oracle.particle_filter(Y, "sir", (1.0, 0.5), False, 0.1, 200, 4820, 20, key=99, filter_index=3)
    u = ph.init_uniforms(99, 3, 0, 200)
    np.testing.assert_array_equal(o["hidden"][0, :, 1], ph.poisson_inversion(u, 20.0))
    assert abs(o["hidden"][0, :, 1].mean() - 20) < 1.5


def test_oracle_systematic_resampling_runs():
    Y = np.load(__import__("os").path.join(__import__("conftest").GOLDEN, "datasets.npz"))["sir_binom"]
    o = oracle.particle_filter(Y, "sir", (2.0, 1.0), False, 0.1, 64, 4820, 20, key=5, filter_index=0,
                               resample="systematic")
    assert o["status"] == 0
    # systematic ancestors are non-decreasing in j
    assert np.all(np.diff(o["ancestry"][1:], axis=1) >= 0)


def test_oracle_binom_pmf_is_the_true_pmf_to_an_ulp():
    """The compensated weight (binary128 log-factorials, hi + lo log; the device runs the same operations) against
    200-bit truth: within 2 ulps everywhere, n up to 2e5, bulk and tails (scripts/scipy_pmf_envelope.py measures
    scipy's own error, up to ~1e-11, on the same kind of sample)."""
    import mpmath
    mpmath.mp.prec = 200
    rs = np.random.RandomState(3)
    M = 1500
    n = np.floor(np.exp(rs.uniform(0, np.log(2e5), M))).astype(np.int64)
    p = np.where(rs.rand(M) < 0.5, 0.1, rs.uniform(0.001, 0.999, M))
    k = np.clip(np.round(n * p + rs.randn(M) * 6 * np.sqrt(n * p * (1 - p))), 0, n).astype(np.int64)
    got = oracle.binom_pmf(k, n, p)
    worst = 0.0
    for i in range(M):
        P = mpmath.mpf(float(p[i]))
        tru = mpmath.binomial(int(n[i]), int(k[i])) * P ** int(k[i]) * (1 - P) ** int(n[i] - k[i])
        if tru < mpmath.mpf("1e-300"):
            continue
        worst = max(worst, abs(float(mpmath.mpf(float(got[i])) / tru - 1)))
    assert worst <= 2 * 2.0 ** -52, worst
