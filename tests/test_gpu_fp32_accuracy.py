"""Elementwise accuracy of the fp32 Johnson layer (north star: fp32 rtol 1e-5).

The reference computes y = gamma + delta*asinh((x - xi)/lambda) in the data precision
(src/johnson_trafo.jl:29-32); Julia's asinh(::Float32) is accurate to a few ulp for every z,
including |z| << 1 where it switches to the log1p form. These tests hold the kernels to that,
elementwise, where tests/parity.py's column-normwise criterion would hide a small-|z| error:

* a single JohnsonTrafo with gamma = xi = 0 (y = delta*asinh(x/lambda)) over |x| in 1e-30 .. 3e38,
  on every kernel family (fragment interpreter D = 2 / 32, LDS-staged generic kernel D = 5,
  the compiled (J o H)^n program), against np.arcsinh in float64 of the same fp32 inputs;
* the config-3 flow (J o H)^4 with gamma = xi = 0 on columns scaled to 1e-30 .. 1 (the flow is
  then ~linear and every intermediate value is tiny: relative accuracy must hold through every
  layer, not only the last);
* the config-3 flow with the survey's parameter distributions, per element
  with the per-element scale |gamma_n| + |delta_n*asinh(z_n)| = |gamma_n| + |y_hi - gamma_n|
  (SURVEY.md §7 "Parity criterion"); where z_n itself cancels (z_n = (u - xi)/lambda with u the
  last reflection's output, both O(1)) no fp32 evaluation, the reference's included, has that
  accuracy, and the bound there is the rounding bound of the last layer's inputs: the reflection's
  D-term dot product alone carries up to D ulps of sum|vh y_prev| (Higham's gamma_D), the kernel
  multiplies by the precomputed 1/lambda, xi/lambda, vh/lambda where the reference divides (three
  more roundings), and y_prev carries the earlier layers' errors, so
  2 (D + 8) * 2^-24 * delta/(lambda sqrt(1+z^2)) * (|y_prev| + |vh| sum|vh y_prev| + |xi|), or 4x the
  reference fp32 algorithm's own error on that element (it also exceeds the conditioning bound on a
  few elements: errors of the earlier layers enter y_prev); over all such elements the kernel's RMS
  error is within 2x the reference's.
"""
from __future__ import annotations

import numpy as np
import pytest

from parity import col_err, colmajor_cuda, make_flow, rand_params, to_np

pytestmark = pytest.mark.gpu

RTOL32 = 1e-5


def wide_values(rng):
    v = np.concatenate([np.logspace(-30, 30, 4000), np.logspace(30, 38.5, 200), rng.uniform(0, 0.25, 3000),
                        rng.standard_normal(2000) * 3,
                        [0.0, 1e-38, 1e-20, 2.44e-4, 0.0625, 0.125, 0.12499999, 0.12500001, 1.0, 1e18, 2e18,
                         3e38, np.inf, np.nan]]).astype(np.float32)
    return np.concatenate([v, -v])


def elem_rel_err(Y, ref):
    fin = np.isfinite(ref) & (ref != 0)
    return float(np.max(np.abs(Y[fin].astype(np.float64) - ref[fin]) / np.abs(ref[fin])))


@pytest.mark.parametrize("D", [2, 32, 5])
def test_fp32_asinh_wide_range(enf, gpu, D):
    """y = asinh(x) (gamma = xi = 0, delta = lambda = 1) elementwise within 1e-5 (measured ~1e-6),
    with signed zeros, Inf and NaN as the reference."""
    rng = np.random.default_rng(7)
    v = wide_values(rng)
    n = (v.size + D - 1) // D * D
    x = np.zeros(n, np.float32)
    x[:v.size] = v
    X = np.asfortranarray(x.reshape(-1, D).T)
    one, zero = np.ones(D, np.float32), np.zeros(D, np.float32)
    layers = [(3, [zero, one, zero, one])]
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y = to_np(Y)
    ref = 0.0 + np.arcsinh(X.astype(np.float64))  # gamma + delta*asinh: 0 + (-0) is +0, as in the reference
    err = elem_rel_err(Y, ref)
    assert err <= 2e-6, f"asinh relative error {err:.3e}"
    assert np.array_equal(np.isnan(Y), np.isnan(ref))
    inf = np.isinf(ref)
    assert np.array_equal(Y[inf], ref[inf].astype(np.float32))
    zero_ = ref == 0
    assert np.array_equal(np.signbit(Y[zero_]), np.signbit(ref[zero_]))


def test_fp32_asinh_scaled_delta_lambda(enf, gpu):
    """The same through delta, lambda != 1 (y = delta*asinh(x/lambda), folded constants of the
    fragment kernel: delta*ln2, 1/lambda), D = 32, against the float64 evaluation of the fp32
    reference formula on the same fp32 inputs."""
    rng = np.random.default_rng(8)
    D, N = 32, 4096
    X = (rng.standard_normal((D, N)) * 10.0 ** rng.uniform(-30, 1, (D, N))).astype(np.float32)
    X = np.asfortranarray(X)
    zero = np.zeros(D, np.float32)
    d, lam = rng.uniform(0.5, 2, D).astype(np.float32), rng.uniform(0.5, 2, D).astype(np.float32)
    layers = [(3, [zero, d, zero, lam])]
    Y = to_np(enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))[0])
    z = X.astype(np.float64) / lam.astype(np.float64)[:, None]
    ref = d.astype(np.float64)[:, None] * np.arcsinh(z)
    err = elem_rel_err(Y, ref)
    assert err <= 3e-6, f"relative error {err:.3e}"


def hj_layers(rng, D, pairs, homogeneous):
    layers = []
    for _ in range(pairs):
        layers.append((5, [rng.standard_normal(D).astype(np.float32)]))
        g, d, xi, lam = rand_params(rng, 3, D, np.float32)
        if homogeneous:
            g, xi = np.zeros_like(g), np.zeros_like(xi)
        layers.append((3, [g, d, xi, lam]))
    return layers


@pytest.mark.parametrize("D,pairs", [(32, 4), (32, 1), (64, 4)])
def test_fp32_flow_homogeneous_tiny(enf, gpu, oracle, D, pairs):
    """(J o H)^n with gamma = xi = 0 on columns scaled by 10^U(-30, 0): relative (column-normwise)
    accuracy through every layer of the compiled program. With asinh's absolute-error fast form
    the tiny columns would come out with errors ~1e-7 absolute, i.e. 1e23 relative."""
    rng = np.random.default_rng(10 + D + pairs)
    N = 20_011
    layers = hj_layers(rng, D, pairs, homogeneous=True)
    X = rng.standard_normal((D, N)) * 10.0 ** rng.uniform(-30, 0, N)[None, :]
    X = np.asfortranarray(X.astype(np.float32))
    Y, L = enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))
    Y, L = to_np(Y), to_np(L).reshape(-1)
    Yh, Lh = oracle.flow_apply_hi(layers, X)
    Yr, _ = oracle.flow_apply(layers, X, nthreads=8)
    ey, ey_ref = col_err(Y, Yh), col_err(Yr, Yh)
    assert ey <= RTOL32, f"column-normwise error {ey:.3e} (reference fp32 {ey_ref:.3e})"
    assert np.all(np.abs(L - Lh) <= RTOL32 * (np.abs(Lh) + 1))


@pytest.mark.parametrize("D", [32, 64])
def test_fp32_flow_per_element(enf, gpu, oracle, D):
    """Config-3 flow (J o H)^4, survey parameter distributions: every output element within
    1e-5 * (|gamma_n| + |delta_n asinh z_n|) of the high-precision value, or within the rounding
    bound of the last layer's inputs where z_n cancels (module docstring)."""
    rng = np.random.default_rng(3 * D)
    N = 100_003
    layers = hj_layers(rng, D, 4, homogeneous=False)
    X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
    Y = to_np(enf.with_logabsdet_jacobian(make_flow(enf, layers), colmajor_cuda(X))[0]).astype(np.float64)
    Yh, _ = oracle.flow_apply_hi(layers, X)
    Yp, _ = oracle.flow_apply_hi(layers[:-2], X)  # input of the last reflection
    v = layers[-2][1][0].astype(np.float64)
    vh = v * np.sqrt(2.0 / (v @ v))
    g, d, xi, lam = (p.astype(np.float64)[:, None] for p in layers[-1][1])
    u = Yp - vh[:, None] * (vh @ Yp)[None, :]
    z = (u - xi) / lam
    cond = d / (lam * np.sqrt(1 + z * z)) * (np.abs(Yp) + np.abs(vh)[:, None] * (np.abs(vh) @ np.abs(Yp))[None, :]
                                             + np.abs(xi))
    Yr, _ = oracle.flow_apply(layers, X, nthreads=8)
    scale = np.abs(g) + np.abs(Yh - g)
    err, err_ref = np.abs(Y - Yh), np.abs(Yr.astype(np.float64) - Yh)
    bound = np.maximum(np.maximum(RTOL32 * scale, 2 * (D + 8) * 2.0 ** -24 * cond), 4 * err_ref)
    ok = err <= bound
    bad = np.argwhere(~ok)
    info = [(tuple(b), f"err {err[tuple(b)]:.2e} ref {err_ref[tuple(b)]:.2e} scale {scale[tuple(b)]:.2e} "
                       f"cond {cond[tuple(b)]:.2e} z {z[tuple(b)]:.2e} y {Yh[tuple(b)]:.2e}") for b in bad[:4]]
    assert ok.all(), f"{bad.shape[0]} elements fail, worst {np.max(err / bound):.2f} x bound; {info}"
    hard = err_ref > RTOL32 * scale  # where the reference itself misses the elementwise bound
    if hard.any():
        rms, rms_ref = np.sqrt(np.mean(err[hard] ** 2)), np.sqrt(np.mean(err_ref[hard] ** 2))
        print(f"D={D}: {hard.sum()} elements where the reference misses 1e-5*scale; RMS error {rms:.3e} vs the "
              f"reference's {rms_ref:.3e}")
        assert rms <= 2 * rms_ref, f"RMS error {rms:.3e} vs reference {rms_ref:.3e} on {hard.sum()} elements"
    # the elementwise criterion proper holds wherever z_n does not cancel
    big = np.abs(z) > 0.25
    assert np.all(err[big] <= RTOL32 * scale[big])
