"""Relative error of the fp32 asinh forms of the fused kernels (enf_frag.h asinh2_*), emulated in
numpy float32 (correctly rounded sqrt, float32 log2 standing in for v_log_f32), against float64
asinh. Forms:
  merge  the Taylor form below kAsinhSmall merged with log2(|z| + sqrt(q)) (asinh2_f32)
  med3   med3(S, -(t + b), t + b): the Taylor form clamped by the biased log form (one v_med3_f32);
         argument "K" (default): the kernel's form, b = log2(K)/2 through z' = sqrt(K) z
Prints the max relative error per |z| decade and overall."""
import sys

import numpy as np

LN2 = np.log(2.0)
A2 = 3.0 / 40.0
A1 = -1.0 / 6.0 - 2.0 * A2
A0 = 1.0 + 1.0 / 6.0 + A2
f32 = np.float32


def taylor(z, q, terms=3):
    if terms == 3:
        p = (q * (q * f32(A2 / LN2) + f32(A1 / LN2)) + f32(A0 / LN2)).astype(f32)
    else:  # 4 terms: z (1 - u/6 + 3u^2/40 - 5u^3/112), u = q - 1, as a cubic in q
        c = np.polynomial.polynomial.Polynomial([1, -1 / 6, 3 / 40, -5 / 112])
        pq = c(np.polynomial.polynomial.Polynomial([-1, 1]))  # in q
        k = pq.coef / LN2
        p = (((q * f32(k[3]) + f32(k[2])) * q + f32(k[1])) * q + f32(k[0])).astype(f32)
    return (z * p).astype(f32)


def forms(z, b, terms):
    z = z.astype(f32)
    q = (z.astype(np.float64) ** 2 + 1.0).astype(f32)
    s = np.sqrt(q).astype(f32)
    w = (np.abs(z) + s).astype(f32)
    t = np.log2(w).astype(f32)
    S = taylor(z, q, 3)
    merge = np.where(t < f32(0.17987053), S, np.copysign(t, z)).astype(f32)
    if b == "K":  # the kernel's form: z' = sqrt(K) z, q' = z'^2 + K, bias log2(K)/2 through the argument
        K = 1.0 + 2.0 ** -21
        zk = (z.astype(np.float64) * np.sqrt(K)).astype(f32)
        qk = (zk.astype(np.float64) ** 2 + K).astype(f32)
        tb = np.log2((np.abs(zk) + np.sqrt(qk).astype(f32)).astype(f32)).astype(f32)
        rk = 1.0 / np.sqrt(K) / LN2
        p = (qk * (qk * f32(A2 * rk / K ** 2) + f32(A1 * rk / K)) + f32(A0 * rk)).astype(f32)
        S2 = (zk * p).astype(f32)
    else:
        S2 = taylor(z, q, terms)
        tb = (t + f32(b)).astype(f32)
    med = np.clip(S2, -tb, tb).astype(f32)
    return merge, med


def main():
    b = sys.argv[1] if len(sys.argv) > 1 else "K"
    b = b if b == "K" else float(b)
    terms = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rng = np.random.default_rng(0)
    e = rng.uniform(-30, 3, 4_000_000)
    z = (10.0 ** e * np.where(rng.random(e.size) < 0.5, -1, 1)).astype(f32)
    ref = np.arcsinh(z.astype(np.float64)) / LN2
    merge, med = forms(z, b, terms)
    rm = np.abs(merge - ref) / np.abs(ref)
    rd = np.abs(med - ref) / np.abs(ref)
    az = np.abs(z.astype(np.float64))
    print(f"b = {b}, taylor terms = {terms}")
    for lo in range(-30, 3):
        m = (az >= 10.0 ** lo) & (az < 10.0 ** (lo + 1))
        if lo < -8 and lo % 5:
            continue
        print(f"|z| in [1e{lo}, 1e{lo + 1}): merge {rm[m].max():.2e}  med3 {rd[m].max():.2e}  "
              f"med3 mean signed {((med - ref) / np.abs(ref))[m].mean():+.1e}")
    print(f"overall max: merge {rm.max():.2e} med3 {rd.max():.2e}")


if __name__ == "__main__":
    main()
