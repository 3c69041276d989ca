"""Dense-Householder (chained HouseholderTrafo) throughput: one JSON line per
(dtype, D, k) with samples/s and algorithmic GB/s ((2D+1)*sizeof(T) per sample). Run it once as is
(MFMA kernel for k >= 8) and once with ENF_WY_MIN_K=100000 (reflection-by-reflection interpreter)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enf_pkg import load  # noqa: E402


def main():
    enf = load()
    torch.cuda.set_device(0)
    path = "interp" if int(os.environ.get("ENF_WY_MIN_K", "8")) > 1000 else "mfma"
    cases = [(np.float32, 32, 10_000_000, k) for k in (1, 4, 8, 16, 32)] + \
            [(np.float32, 64, 12_500_000, k) for k in (8, 32, 64)] + \
            [(np.float64, 32, 5_000_000, k) for k in (8, 32)] + [(np.float64, 64, 5_000_000, 64)]
    flows = os.environ.get("WY_FLOWS", "H,JH").split(",")
    for dt, D, N, k in cases:
        rng = np.random.default_rng(42)
        tdt = torch.float32 if dt == np.float32 else torch.float64
        g = torch.Generator(device="cuda").manual_seed(0x5EED)
        X = torch.randn((N, D), device="cuda", generator=g, dtype=tdt).t()
        for fl in flows:
            H = enf.HouseholderTrafo(np.asfortranarray(rng.standard_normal((D, k)).astype(dt)))
            if fl == "H":
                f = H
            else:  # J o H: the elementwise layer in the same launch
                J = enf.JohnsonTrafo(rng.uniform(-1, 1, D).astype(dt), rng.uniform(0.5, 2, D).astype(dt),
                                     rng.uniform(-0.5, 0.5, D).astype(dt), rng.uniform(0.5, 2, D).astype(dt))
                f = enf.compose(J, H)
            for _ in range(3):
                enf.with_logabsdet_jacobian(f, X)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                enf.with_logabsdet_jacobian(f, X)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            bps = (2 * D + 1) * np.dtype(dt).itemsize
            print(json.dumps({"path": path, "flow": fl, "dtype": np.dtype(dt).name, "D": D, "k": k, "N": N,
                              "ms": round(ms, 4), "samples_per_s": N / ms * 1e3,
                              "GBps": N * bps / ms / 1e6, "hbm_frac": N * bps / ms / 1e6 / 8000.0}), flush=True)


if __name__ == "__main__":
    main()
