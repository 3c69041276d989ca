"""GPU parity of the device JohnsonSU distribution (enf_johnsonsu.hip)
against the oracle restatement (oracle/enf_oracle_jsu.c), the exact golden values
(tests/golden/johnsonsu.npz) and the reference's own sampling test (test/test_johnson_trafo.jl:12-14)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FNS = ("pdf", "logpdf", "cdf", "logcdf", "ccdf", "logccdf", "quantile")


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "johnsonsu.npz"))


def _rel_tol(fn, y, base, eps):
    """Error bound of the reference formula in precision eps: the normal argument y carries ~|y| eps,
    which exp(-y^2/2) / Phi(y) turn into ~y^2 eps relative."""
    return base + 8 * eps * (1 + y * y)


@pytest.mark.parametrize("fn", FNS)
def test_jsu_fp64_vs_golden_and_oracle(enf, gpu, oracle, golden, fn):
    import torch

    for i, prm in enumerate(golden["params"]):
        d = enf.JohnsonSU(*[float(v) for v in prm])
        x = golden[f"p{i}"] if fn == "quantile" else golden[f"x{i}"]
        got = d._eval(fn, torch.from_numpy(x).cuda()).cpu().numpy()
        ref = oracle.jsu_eval(fn, x, *prm)
        g, de, xi, l = prm
        if fn == "quantile":
            assert np.allclose(got, ref, rtol=1e-12, atol=1e-15), (i, fn)
            assert np.allclose(got, golden[f"quantile{i}"], rtol=1e-12, atol=1e-15), (i, fn)
            continue
        y = g + de * np.arcsinh((x - xi) / l)
        tol = _rel_tol(fn, y, 1e-13, 2.2e-16)
        if fn in ("ccdf", "logccdf"):  # 1 - cdf: absolute in the complement
            cc = golden[f"ccdf{i}"]
            err = np.where(got == ref, 0.0, np.abs(got - ref)) * (cc if fn == "logccdf" else 1.0)
            assert (err <= 4e-15 + 1e-15 * cc).all(), (i, fn)
            continue
        scale = np.maximum(np.abs(ref), 1e-3) if fn == "logcdf" else np.abs(ref)
        assert (np.abs(got - ref) <= tol * scale + 1e-300).all(), (i, fn, np.max(np.abs(got - ref) / scale))
        exact = golden[f"{fn}{i}"]
        assert (np.abs(got - exact) <= tol * (np.maximum(np.abs(exact), 1e-3) if fn == "logcdf" else np.abs(exact))
                + 1e-300).all(), (i, fn)


@pytest.mark.parametrize("fn", FNS)
def test_jsu_fp32_vs_oracle(enf, gpu, oracle, fn):
    """Float32 parameters and data (Julia keeps Float32): against the oracle in double at the same
    float32 inputs, |y| <= 8."""
    import torch

    rng = np.random.default_rng(3)
    for prm in ((-1.5, 1.5, 0.5, 2.0), (0.3, 1.0, -4.0, 0.5), (2.0, 3.5, 1.0, 1.0)):
        p32 = [np.float32(v) for v in prm]
        d = enf.JohnsonSU(*p32)
        assert d.partype == np.float32
        if fn == "quantile":
            x = rng.uniform(1e-6, 1 - 1e-6, 20000).astype(np.float32)
        else:
            y = rng.uniform(-8, 8, 20000)
            x = (p32[3] * np.sinh((y - p32[0]) / p32[1]) + p32[2]).astype(np.float32)
        got = d._eval(fn, torch.from_numpy(x).cuda())
        assert got.dtype == torch.float32
        got = got.cpu().numpy().astype(np.float64)
        ref = oracle.jsu_eval(fn, x.astype(np.float64), *[float(v) for v in p32])
        if fn == "quantile":
            # sinh((z - g)/d) amplifies the float32 rounding of z by |w coth w|, w = (z - g)/d
            z = np.sqrt(2) * __import__("scipy.special", fromlist=["erfinv"]).erfinv(2 * x.astype(np.float64) - 1)
            w = (z - p32[0]) / p32[1]
            cond = 1 + np.abs(w / np.tanh(np.where(w == 0, 1e-30, w))) * (1 + np.abs(z))
            assert (np.abs(got - ref) <= 2e-6 * cond * (np.abs(ref) + p32[3])).all()
            continue
        yy = p32[0] + p32[1] * np.arcsinh((x - p32[2]) / p32[3])
        tol = _rel_tol(fn, yy, 1e-5, 6e-8)
        if fn in ("ccdf", "logccdf", "logcdf"):
            cc = 1 - oracle.jsu_eval("cdf", x.astype(np.float64), *[float(v) for v in p32])
            c = 1 - cc
            if fn == "ccdf":
                assert (np.abs(got - ref) <= 1e-6 + tol * np.abs(ref)).all()
            elif fn == "logccdf":
                m = cc > 1e-3
                assert (np.abs(got - ref)[m] <= (1e-6 + tol[m] * cc[m]) / cc[m]).all()
            else:
                assert (np.abs(got - ref) <= tol * np.maximum(np.abs(ref), 1e-3) + 1e-6 / np.maximum(c, 1e-30)).all()
            continue
        scale = np.maximum(np.abs(ref), 1.0) if fn == "logpdf" else np.abs(ref)  # logs: absolute near 0
        assert (np.abs(got - ref) <= tol * scale + 1e-37).all(), (fn, np.max(np.abs(got - ref) / scale))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_jsu_sampler_vs_oracle_stream(enf, gpu, oracle, dtype):
    """rand(d, n) = quantile(d, u) with the documented Philox4x32-10 uniforms: the device draws equal
    the oracle's quantile of the oracle's uniform stream; sharding by offset reproduces one draw."""
    prm = (-15.0, 6.5, 0.0, 2.5)
    d = enf.JohnsonSU(*(dtype(v) for v in prm)) if dtype == np.float32 else enf.JohnsonSU(*prm)
    n, seed = 100_003, 0x5EED
    s = d.rand(n, seed=seed).cpu().numpy()
    assert s.dtype == dtype and np.isfinite(s).all()
    u = oracle.jsu_uniforms(dtype, n, seed)
    ref = oracle.jsu_eval("quantile", u, *prm)
    rtol = 1e-12 if dtype == np.float64 else 2e-5
    assert np.allclose(s, ref, rtol=rtol, atol=rtol * 2.5), np.max(np.abs(s - ref))
    per = 4 if dtype == np.float32 else 2
    part = d.rand(1000, seed=seed, offset=5000 // per).cpu().numpy()
    assert np.array_equal(part, s[5000:6000])
    assert np.array_equal(d.rand(n, seed=seed).cpu().numpy(), s)
    assert not np.array_equal(d.rand(1000, seed=seed + 1).cpu().numpy(), s[:1000])


def test_jsu_reference_sampling_test(enf, gpu):
    """test/test_johnson_trafo.jl:12-14: mean |sorted x| of rand(JohnsonSU(-15, 6.5, 0, 2.5), 10^6)
    matches johnsontrafo_inv.(randn(10^6), -15, 6.5, 0, 2.5) at rtol 0.01 (the latter through the
    JohnsonTrafoInv flow kernel)."""
    import torch

    n = 10 ** 6
    X = enf.JohnsonSU(-15, 6.5, 0, 2.5).rand(n, seed=1)
    g = torch.Generator(device="cuda").manual_seed(2)
    K = torch.randn((1, n), device="cuda", dtype=torch.float64, generator=g)
    one = lambda v: np.array([v], dtype=np.float64)
    Kj = enf.JohnsonTrafoInv(one(-15), one(6.5), one(0), one(2.5))(K)
    a = float(torch.sort(Kj.abs().reshape(-1)).values.sum()) / n
    b = float(torch.sort(X.abs()).values.sum()) / n
    assert abs(a - b) <= 0.01 * max(a, b)


def test_jsu_sampler_distribution(enf, gpu, oracle):
    """Kolmogorov-Smirnov distance of 4e6 fp64 draws from the oracle cdf, sample mean and variance
    against the reference's mean / var (src/johnson_trafo.jl:24,26)."""
    d = enf.JohnsonSU(0.5, 1.7, -1.0, 2.0)
    n = 4_000_000
    s = np.sort(d.rand(n, seed=11).cpu().numpy())
    F = oracle.jsu_eval("cdf", s, 0.5, 1.7, -1.0, 2.0)
    ks = max(np.max(np.arange(1, n + 1) / n - F), np.max(F - np.arange(n) / n))
    assert ks < 1.63 / np.sqrt(n)  # 1 % level
    assert abs(s.mean() - d.mean()) < 5 * np.sqrt(d.var() / n)
    assert abs(s.var() / d.var() - 1) < 0.01


def test_jsu_host_interface(enf, gpu):
    """Scalars and numpy in, Julia promotion (Float32 data with Float64 parameters -> Float64),
    statistics, errors."""
    import torch

    d = enf.JohnsonSU()  # keyword defaults of johnson_trafo.jl:9-12
    assert (d.gamma, d.delta, d.xi, d.lambda_) == (10.0, 3.5, 10.0, 1.0)
    v = d.pdf(10.5)
    assert isinstance(v, np.float64) and v > 0
    out = d.cdf(np.array([-5.0, 1.3, 5.0], dtype=np.float32))  # y = 10 + 3.5 asinh(x - 10) around 0
    assert out.dtype == np.float64 and np.all(np.diff(out) > 0)
    assert d.location() == d.mean() and d.scale() == d.var()
    assert d.quantile(0.5) == pytest.approx(d.median(), rel=1e-12)
    with pytest.raises(enf.MethodError):
        d.pdf(torch.zeros(3))  # host tensor
    with pytest.raises(enf.MethodError):
        enf.JohnsonSU(np.ones(2), 1.0, 0.0, 1.0)
    assert d.rand(0).numel() == 0
