"""JohnsonSU on the device: throughput of rand (Philox + quantile) and of
the elementwise logpdf / cdf / quantile over 1e8 values, one JSON line each. Bytes per value:
sizeof(T) written (rand), 2 sizeof(T) read + written (eval)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enf_pkg import load  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    enf = load()
    torch.cuda.set_device(0)
    n = int(os.environ.get("JSU_N", "100000000"))
    for dt in (np.float32, np.float64):
        d = enf.JohnsonSU(*(dt(v) for v in (-15.0, 6.5, 0.0, 2.5)))
        sz = np.dtype(dt).itemsize
        ms = timed(lambda: d.rand(n, seed=1))
        print(json.dumps({"what": "rand", "dtype": np.dtype(dt).name, "n": n, "ms": round(ms, 4),
                          "values_per_s": n / ms * 1e3, "GBps": n * sz / ms / 1e6}), flush=True)
        x = d.rand(n, seed=2)
        p = torch.rand(n, device="cuda", dtype=x.dtype)
        for fn, arg in (("logpdf", x), ("cdf", x), ("quantile", p)):
            ms = timed(lambda: d._eval(fn, arg))
            print(json.dumps({"what": fn, "dtype": np.dtype(dt).name, "n": n, "ms": round(ms, 4),
                              "values_per_s": n / ms * 1e3, "GBps": 2 * n * sz / ms / 1e6}), flush=True)
        del x, p


if __name__ == "__main__":
    main()
