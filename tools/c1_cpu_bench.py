"""Config 1 (ScaleShiftTrafo D=1, N=1e3 fp64 on CPU, no GPU): libenf's host path
(enf_flow_apply_cpu through the mirror's with_logabsdet_jacobian on a numpy batch) timed per call,
with the oracle's reference-structured restatement of the same call beside it. Also a larger host
batch (D = 32, N = 1e6, (J o H)^4 fp64) to show the threaded path's throughput. One JSON line each."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def timeit(fn, min_s=1.0):
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= min_s:
            return dt / n


def main():
    from enf_pkg import load
    import bench
    import oracle  # checker / baseline only

    enf = load()
    rng = np.random.default_rng(1)
    X = rng.standard_normal((1, 1000))
    a, b = np.array([-1.7]), np.array([0.25])
    f = enf.ScaleShiftTrafo(a, b)
    layers = [(0, [a, b])]
    t_enf = timeit(lambda: enf.with_logabsdet_jacobian(f, X))
    t_orc = timeit(lambda: oracle.flow_apply(layers, X))
    Y, L = enf.with_logabsdet_jacobian(f, X)
    Yr, Lr = oracle.flow_apply(layers, X)
    print(json.dumps({"config": "C1 ScaleShiftTrafo D=1 N=1e3 fp64, host data", "path": "enf_flow_apply_cpu via mirror",
                      "us_per_call": t_enf * 1e6, "oracle_us_per_call": t_orc * 1e6,
                      "max_abs_diff_vs_oracle": float(np.abs(Y - Yr).max()), "ladj_equal": bool(np.array_equal(L[0], Lr))}))
    D, N = 32, 1_000_000
    fl = bench.build_flow(D, 4, np.float64)
    F = enf.compose(*[enf.HouseholderTrafo(ps[0]) if op == 5 else enf.JohnsonTrafo(*ps) for op, ps in reversed(fl)])
    Xb = np.asfortranarray(rng.standard_normal((D, N)))
    t_big = timeit(lambda: enf.with_logabsdet_jacobian(F, Xb), 2.0)
    print(json.dumps({"config": "C3 flow fp64 on host data, D=32 N=1e6", "path": "enf_flow_apply_cpu, all threads",
                      "threads": os.cpu_count(), "samples_per_s": N / t_big, "ms_per_call": t_big * 1e3}))


if __name__ == "__main__":
    main()
