"""CPU: the oracle's JohnsonSU distribution functions (src/johnson_trafo.jl:120-129, restated in
oracle/enf_oracle_jsu.c) pinned by the exact mpmath golden values (tests/golden/johnsonsu.npz,
oracle/gen_golden.py), and its Philox4x32-10 stream pinned by the Random123 known-answer vectors."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

FNS = ("pdf", "logpdf", "cdf", "logcdf", "ccdf", "logccdf")


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "johnsonsu.npz"))


def test_philox_known_answers(oracle):
    """Random123's philox4x32-10 KATs (Salmon et al., SC'11; kat_vectors)."""
    assert oracle.philox4x32_10((0, 0, 0, 0), (0, 0)) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert oracle.philox4x32_10((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2) == (0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                          0x6D5451FD)
    assert oracle.philox4x32_10((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == \
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


@pytest.mark.parametrize("fn", FNS)
def test_jsu_functions_vs_golden(oracle, golden, fn):
    """Relative 1e-13 where the reference formula is well conditioned; ccdf / logccdf follow the
    reference's 1 - cdf (src/johnson_trafo.jl:125-126), exact to a few 1e-15 absolute in 1 - cdf."""
    for i, (g, d, xi, l) in enumerate(golden["params"]):
        x = golden[f"x{i}"]
        got = oracle.jsu_eval(fn, x, g, d, xi, l)
        exact = golden[f"{fn}{i}"]
        if fn in ("ccdf", "logccdf"):
            cc = golden[f"ccdf{i}"]
            ok = np.abs(oracle.jsu_eval("ccdf", x, g, d, xi, l) - cc) <= 4e-15 + 1e-15 * cc
            assert ok.all(), (i, fn)
            if fn == "logccdf":  # where 1 - cdf keeps relative precision
                m = cc > 1e-3
                assert (np.abs(got[m] - exact[m]) <= (4e-15 + 1e-15 * cc[m]) / cc[m]).all(), (i, fn)
            continue
        # the standard-normal argument y carries ~|y| eps of rounding, which exp(-y^2/2) and Phi(y)
        # turn into ~y^2 eps relative: the reference formula's own conditioning
        y = g + d * np.arcsinh((x - xi) / l)
        rel = 1e-13 + 8e-16 * (1 + y * y)
        if fn == "logcdf":
            tol = rel * np.maximum(np.abs(exact), 1e-3)
        else:
            tol = rel * np.abs(exact) + (1e-300 if fn == "pdf" else 0)
        assert (np.abs(got - exact) <= tol).all(), (i, fn, np.max(np.abs(got - exact) / np.abs(exact)))


def test_jsu_quantile_vs_golden(oracle, golden):
    for i, (g, d, xi, l) in enumerate(golden["params"]):
        p = golden[f"p{i}"]
        got = oracle.jsu_eval("quantile", p, g, d, xi, l)
        exact = golden[f"quantile{i}"]
        # sinh amplifies the normal quantile's rounding by |(z - g)/d| coth(...): 1e-12 relative
        assert np.allclose(got, exact, rtol=1e-12, atol=1e-15), (i, np.max(np.abs(got - exact) / np.abs(exact)))


def test_jsu_cdf_quantile_round_trip(oracle):
    p = np.linspace(1e-6, 1 - 1e-6, 1001)
    for prm in ((-15.0, 6.5, 0.0, 2.5), (0.4, 1.3, 2.0, 0.7)):
        x = oracle.jsu_eval("quantile", p, *prm)
        assert np.allclose(oracle.jsu_eval("cdf", x, *prm), p, rtol=1e-12, atol=1e-15)


def test_jsu_uniform_stream(oracle):
    """The sampler's uniforms: in (0, 1), 4 (fp32) / 2 (fp64) per Philox call, offset = calls."""
    u32 = oracle.jsu_uniforms(np.float32, 4000, seed=7)
    u64 = oracle.jsu_uniforms(np.float64, 4000, seed=7)
    for u in (u32, u64):
        assert (u > 0).all() and (u < 1).all()
        assert abs(u.mean() - 0.5) < 0.02
    assert np.array_equal(oracle.jsu_uniforms(np.float32, 400, seed=7, offset=100), u32[400:800])
    assert np.array_equal(oracle.jsu_uniforms(np.float64, 400, seed=7, offset=100), u64[200:600])
    assert np.all(u32 == u32.astype(np.float32))  # exactly the device's fp32 values
