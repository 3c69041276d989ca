"""Shared parity criteria and helpers for the tests.

Why normwise per column: a Householder output component and a Johnson `gamma + delta*asinh(z)`
can cancel to ~0, and then NO fixed-precision evaluation -- the reference's own included -- has a
small elementwise relative error (the reference's fp32 path shows 6e-4 elementwise against the
exact values, tests/golden; SURVEY.md §7 "Parity criterion"). The criterion is therefore
    |y - y_ref| <= rtol * (|y_ref| + max_d |y_ref[:, j]|)           for outputs (column j),
    |l - l_ref| <= rtol * (|l_ref| + 1)                              for ladj,
with the north-star tolerances rtol = 1e-12 (fp64) and 1e-5 (fp32).

Where the reference algorithm itself cannot meet that bound in its own precision T (a D = 1 or 2
column whose entries all cancel to ~0), the bound is "no worse than K = 4 times the reference's own
error": errors are measured against a higher-precision evaluation of the same formulas on the same
rounded inputs (oracle.flow_apply_hi: fp32 -> float64, fp64 -> x87 extended; or the exact mpmath
golden values), and a result passes if
    err(gpu) <= max(rtol, K * err(reference in T)).
"""
from __future__ import annotations

import numpy as np

RTOL = {np.dtype(np.float64): 1e-12, np.dtype(np.float32): 1e-5}


def to_np(t):
    import torch

    if isinstance(t, torch.Tensor):
        return t.detach().cpu().numpy()
    return np.asarray(t)


def col_err(Y, Yref):
    Y = np.asarray(Y, dtype=np.float64)
    Yref = np.asarray(Yref, dtype=np.float64)
    if Y.size == 0:
        return 0.0
    scale = np.abs(Yref) + np.abs(Yref).max(axis=0, keepdims=True)
    both_nan = np.isnan(Y) & np.isnan(Yref)
    same_inf = np.isinf(Y) & (Y == Yref)
    with np.errstate(invalid="ignore", divide="ignore"):
        e = np.abs(Y - Yref) / np.where(scale > 0, scale, 1.0)
    e = np.where(both_nan | same_inf, 0.0, e)
    return float(np.nanmax(np.where(np.isnan(e), np.inf, e)))


def ladj_err(L, Lref):
    L = np.asarray(L, dtype=np.float64).reshape(-1)
    Lref = np.asarray(Lref, dtype=np.float64).reshape(-1)
    if L.size == 0:
        return 0.0
    both_nan = np.isnan(L) & np.isnan(Lref)
    same_inf = np.isinf(L) & (L == Lref)
    with np.errstate(invalid="ignore"):
        e = np.abs(L - Lref) / (np.abs(Lref) + 1.0)
    e = np.where(both_nan | same_inf, 0.0, e)
    return float(np.nanmax(np.where(np.isnan(e), np.inf, e)))


def loss_close(got, ref, rtol):
    """A scalar loss against the reference's: equal infinities (an overflowing flow in both) pass, NaN never does,
    finite values within rtol * (|ref| + 1). (Plain |got - ref| <= tol cannot tell a matching +-Inf from a real
    mismatch: Inf - Inf is NaN and the comparison is False either way.)"""
    got, ref = float(got), float(ref)
    if np.isinf(ref) or np.isinf(got):
        return got == ref
    return bool(np.isfinite(got) and np.isfinite(ref) and abs(got - ref) <= rtol * (abs(ref) + 1.0))


K_REF = 4.0


def assert_flow_close(Y, L, Yref, Lref, dtype, factor=1.0, what=""):
    """Plain bound: normwise error of (Y, L) against (Yref, Lref) within rtol*factor."""
    rtol = RTOL[np.dtype(dtype)] * factor
    ey = col_err(Y, Yref)
    assert ey <= rtol, f"{what}: Y normwise error {ey:.3e} > {rtol:.1e}"
    if L is not None:
        el = ladj_err(L, Lref)
        assert el <= rtol, f"{what}: ladj error {el:.3e} > {rtol:.1e}"


def assert_as_accurate(Y, L, Yt, Lt, Yhi, Lhi, dtype, factor=1.0, what=""):
    """(Y, L): result under test; (Yt, Lt): the reference algorithm in the same precision (oracle);
    (Yhi, Lhi): high-precision values. Pass if within rtol of Yhi or no worse than K_REF x the
    reference's own error (see module docstring). Returns the measured errors."""
    rtol = RTOL[np.dtype(dtype)] * factor
    ey, ey_ref = col_err(Y, Yhi), col_err(Yt, Yhi)
    assert ey <= max(rtol, K_REF * ey_ref), (f"{what}: Y error {ey:.3e} > max(rtol {rtol:.1e}, "
                                             f"{K_REF} x reference's own {ey_ref:.3e})")
    el = el_ref = 0.0
    if L is not None:
        el, el_ref = ladj_err(L, Lhi), ladj_err(Lt, Lhi)
        assert el <= max(rtol, K_REF * el_ref), (f"{what}: ladj error {el:.3e} > max(rtol {rtol:.1e}, "
                                                 f"{K_REF} x reference's own {el_ref:.3e})")
    return ey, ey_ref, el, el_ref


def check_vs_oracle(oracle, layers, X, Y, L, dtype, factor=1.0, what=""):
    """Run the oracle in T and in high precision on (layers, X) and apply assert_as_accurate."""
    Yt, Lt = oracle.flow_apply(layers, X, nthreads=8)
    Yhi, Lhi = oracle.flow_apply_hi(layers, X)
    return assert_as_accurate(Y, L, Yt, Lt, Yhi, Lhi, dtype, factor, what)


def rand_params(rng, op, D, dtype, K=1):
    """Synthetic parameter distributions of SURVEY.md §8(d) (same as oracle/gen_golden.py)."""
    u = lambda lo, hi: rng.uniform(lo, hi, D).astype(dtype)
    if op == 0:
        return [(np.where(rng.random(D) < 0.5, -1, 1) * rng.uniform(0.5, 2, D)).astype(dtype),
                rng.standard_normal(D).astype(dtype)]
    if op in (1, 2):
        return [u(0, 2), u(0.5, 2), u(-0.5, 0.5)]
    if op in (3, 4):
        return [u(-1, 1), u(0.5, 2), u(-0.5, 0.5), u(0.5, 2)]
    if op == 5:
        return [np.asfortranarray(rng.standard_normal((D, K)).astype(dtype))]
    raise ValueError(op)


def make_trafo(enf, op, params):
    cls = [enf.ScaleShiftTrafo, enf.CenterStretch, enf.CenterContract, enf.JohnsonTrafo,
           enf.JohnsonTrafoInv, enf.HouseholderTrafo][op]
    if op == 5:
        V = np.asarray(params[0])
        return cls(V if V.ndim == 2 and V.shape[1] > 1 else V.reshape(-1))
    return cls(*params)


def make_flow(enf, layers):
    """Oracle layer list (innermost first) -> composed host trafo."""
    return enf.compose(*[make_trafo(enf, op, ps) for op, ps in reversed(layers)])


def colmajor_cuda(Xh, device="cuda"):
    """numpy (D, N) -> column-major CUDA tensor of shape (D, N)."""
    import torch

    return torch.from_numpy(np.ascontiguousarray(np.asarray(Xh).T)).to(device).t()
