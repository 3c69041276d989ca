"""CPU emulation of the compiled (J o H)^n program's fp32 arithmetic (design tool, not product).

Emulates, operation by operation, two forms of the fp32 pair loop of enf_hj.h on numpy float32 arrays
(fma(a, b, c) = round32(a*b + c) in float64, exact for the product; hardware sqrt / log2 as correctly
rounded float32 of the float64 value):
  * "base": the round-5 product form: y = gamma + delta' L, dot = vh'y, u = y - dot vh, z = u/lambda - xi/lambda
  * "fold": the round-6 form: the interior hop J_{p-1} -> H_p -> J_p folded into per-row constants,
      dot = sum_d w_d L_d      (w = vh delta'_{p-1})
      z   = fma(-dot, c, fma(L, b, a))   (b = delta'/lambda, a = (H gamma - xi)/lambda, c = vh/lambda;
                                          pair 0: w = vh, b = 1/lambda, a = -xi/lambda on x)
and reports the per-element criterion of tests/test_gpu_fp32_accuracy.py::test_fp32_flow_per_element for
each, so the fold can be priced for accuracy before it is built.
Usage: python tools/hj_fold_emul.py [D] [N]
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402

f32 = np.float32
LN2 = np.log(2.0)
A2 = 3.0 / 40.0
A1 = -1.0 / 6.0 - 2.0 * A2
A0 = 1.0 + 1.0 / 6.0 + A2
LOG2E = 1.0 / LN2
QBITS = np.uint32(0x3F820000)
LOG2Q = []  # log2 q of every pair of the last run (the ladj's running product)


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def asinh2(z):
    q = fma(z, z, f32(1.0))
    s = np.sqrt(q.astype(np.float64)).astype(f32)
    w = (np.abs(z).astype(np.float64) + s).astype(f32)  # |z| + s rounds in fp32 first
    t = np.log2(w.astype(np.float64)).astype(f32)
    p = fma(q, fma(q, f32(A2 * LOG2E), f32(A1 * LOG2E)), f32(A0 * LOG2E))
    small = (z * p).astype(f32)
    m = q.view(np.uint32) < QBITS
    L = np.where(m, small, np.copysign(t, z)).astype(f32)
    return L, q


def lane_dot(wrows, Lrows, D, init=None):
    """dot over the D rows of a column as the kernel sums it: R = 8 rows per lane (two chains, even / odd
    rows), G = D/8 lanes combined by the DPP butterfly. wrows: (D,) f32, Lrows: (D, N) f32, init (G,) per-lane
    start of chain 0 (or None: the first product)."""
    R = 8
    G = D // R
    NF = 2
    parts = []
    for g in range(G):
        rows = [h * (D // NF) + 4 * g + e for h in range(NF) for e in range(4)]
        d2 = [None, None]
        for c in range(2):
            r = rows[c]
            if c == 0 and init is not None:
                d2[0] = fma(np.full(1, wrows[r], f32), Lrows[r], np.full(1, init[g], f32))
            else:
                d2[c] = (wrows[r] * Lrows[r]).astype(f32)
        for e in range(2, R):
            r = rows[e]
            d2[e & 1] = fma(np.full(1, wrows[r], f32), Lrows[r], d2[e & 1])
        parts.append((d2[0] + d2[1]).astype(f32))
    # DPP butterfly: quad_perm(1,0,3,2) then (2,3,0,1): ((p0+p1)+(p2+p3)) on every lane
    while len(parts) > 1:
        nxt = []
        for i in range(0, len(parts), 2):
            nxt.append((parts[i] + parts[i + 1]).astype(f32))
        parts = nxt
    return parts[0]


def run(layers, X, form):
    D, N = X.shape
    n = len(layers) // 2
    Vh, G, Dl, Xi, Lm = [], [], [], [], []
    for p in range(n):
        v = layers[2 * p][1][0].astype(np.float64)
        Vh.append(v * np.sqrt(2.0 / (v @ v)))
        g, d, xi, lam = (a.astype(np.float64) for a in layers[2 * p + 1][1])
        G.append(g), Dl.append(d), Xi.append(xi), Lm.append(lam)
    x = X.astype(f32)
    L = None
    LOG2Q.clear()
    for p in range(n):
        vh, il = Vh[p], 1.0 / Lm[p]
        if form == "base":
            if p == 0:
                y = x
            else:
                dp = (Dl[p - 1] * LN2).astype(f32)
                y = fma(L, dp[:, None], G[p - 1].astype(f32)[:, None])
            dot = lane_dot(vh.astype(f32), y, D)
            u = fma(-np.broadcast_to(dot, y.shape), vh.astype(f32)[:, None], y)
            z = fma(u, il.astype(f32)[:, None], (-Xi[p] * il).astype(f32)[:, None])
        else:
            # the folded hop: every pair is dot = W'L, z = fma(-dot, C, fma(L, B, A))
            if p == 0:
                prev, W, B, A = x, vh, il, -Xi[p] * il
            else:
                dpp = Dl[p - 1] * LN2
                hg = G[p - 1] - vh * (vh @ G[p - 1])  # H gamma (double)
                prev, W, B, A = L, vh * dpp, dpp * il, (hg - Xi[p]) * il
            dot = lane_dot(W.astype(f32), prev, D)
            z = fma(prev, B.astype(f32)[:, None], A.astype(f32)[:, None])
            z = fma(-np.broadcast_to(dot, z.shape), (vh * il).astype(f32)[:, None], z)
        L, q = asinh2(z)
        LOG2Q.append(np.log2(q.astype(np.float64)))
    dp = (Dl[n - 1] * LN2).astype(f32)
    return fma(L, dp[:, None], G[n - 1].astype(f32)[:, None])


def per_element(layers, X, Y):
    """tests/test_gpu_fp32_accuracy.py::test_fp32_flow_per_element's criterion; returns (worst err/bound,
    fails, RMS on the hard elements vs the reference's, elementwise fraction within 1e-5 scale)."""
    D = X.shape[0]
    Yh, _ = oracle.flow_apply_hi(layers, X)
    Yp, _ = oracle.flow_apply_hi(layers[:-2], X)
    v = layers[-2][1][0].astype(np.float64)
    vh = v * np.sqrt(2.0 / (v @ v))
    g, d, xi, lam = (p.astype(np.float64)[:, None] for p in layers[-1][1])
    u = Yp - vh[:, None] * (vh @ Yp)[None, :]
    z = (u - xi) / lam
    cond = d / (lam * np.sqrt(1 + z * z)) * (np.abs(Yp) + np.abs(vh)[:, None] * (np.abs(vh) @ np.abs(Yp))[None, :]
                                             + np.abs(xi))
    Yr, _ = oracle.flow_apply(layers, X, nthreads=8)
    scale = np.abs(g) + np.abs(Yh - g)
    err, err_ref = np.abs(Y.astype(np.float64) - Yh), np.abs(Yr.astype(np.float64) - Yh)
    bound = np.maximum(np.maximum(1e-5 * scale, 2 * (D + 8) * 2.0 ** -24 * cond), 4 * err_ref)
    hard = err_ref > 1e-5 * scale
    rms = np.sqrt(np.mean(err[hard] ** 2)) if hard.any() else 0.0
    rms_ref = np.sqrt(np.mean(err_ref[hard] ** 2)) if hard.any() else 0.0
    within = float(np.mean(err <= 1e-5 * scale))
    within_ref = float(np.mean(err_ref <= 1e-5 * scale))
    return float(np.max(err / bound)), int(np.sum(err > bound)), rms, rms_ref, within, within_ref, float(np.max(err / scale))


def main():
    from parity import rand_params

    D = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_003
    for seed in (3 * D, 1, 2):
        rng = np.random.default_rng(seed)
        layers = []
        for _ in range(4):
            layers.append((5, [rng.standard_normal(D).astype(np.float32)]))
            layers.append((3, rand_params(rng, 3, D, np.float32)))
        X = np.asfortranarray(rng.standard_normal((D, N)).astype(np.float32))
        for form in ("base", "fold"):
            Y = run(layers, X, form)
            worst, fails, rms, rms_ref, within, within_ref, wscale = per_element(layers, X, Y)
            # log2 of the running q product of a lane (8 rows of one column, all pairs): the fast path's guard
            lane = sum(lq.reshape(2, D // 8, 4, -1).sum(axis=(0, 2)) for lq in LOG2Q)
            print(f"  running q product: max log2 {lane.max():.1f}, lanes over 128: {(lane > 128).sum()}")
            print(f"seed {seed} D={D} {form}: worst {worst:.3f} x bound, {fails} fail; hard RMS {rms:.3e} vs ref "
                  f"{rms_ref:.3e}; within 1e-5*scale {within:.6f} (ref {within_ref:.6f}); max err/scale {wscale:.2e}")


if __name__ == "__main__":
    main()
