"""A/B timing of one flow configuration on the DIAGNOSTICS library (libenf_diag.so, ENF_DIAG=1):
variants are selected by ENF_* environment knobs (enf_internal.h ENF_KNOB), one process per
variant. Not the benchmark (bench.py times the shipping libenf.so).

    ENF_HJ_ASINH=1 python tools/flow_time.py --D 32 --N 10000000 --pairs 4 --tag fast
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--N", type=int, default=10_000_000)
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--pattern", default=None)
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="run the flow untimed for this long first (the clock ramps over the first ~25 launches)")
    ap.add_argument("--product", action="store_true", help="time the shipping libenf.so instead")
    ap.add_argument("--inverse", action="store_true",
                    help="time inverse(flow) on the forward flow's outputs (bench.py --inverse's workload)")
    ap.add_argument("--lib", default=None, help="time this build of the ABI instead (e.g. tools/ab/libenf_r5.so)")
    ap.add_argument("--flush-mb", type=int, default=0,
                    help="write a buffer of this many MB before every call (evicts the L2s and the MALL: cold-cache "
                         "kernel times under rocprofv3; the event time then includes the writes)")
    args = ap.parse_args()
    from enf_pkg import load
    import bench

    enf = load()
    if args.lib:
        enf._lib.use_diagnostics_library(os.path.join(ROOT, args.lib))
    elif not args.product:
        enf._lib.use_diagnostics_library()
    lib, L = enf._lib, enf._lib.lib()
    dev = torch.device("cuda", 0)
    npd = np.float32 if args.dtype == "f32" else np.float64
    td = torch.float32 if args.dtype == "f32" else torch.float64
    D, N = args.D, args.N
    fwd = bench.build_flow(D, args.pairs, npd, pattern=args.pattern)
    layers = bench.invert_layers(fwd) if args.inverse else fwd
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    X = torch.randn((N, D), generator=g, device=dev, dtype=td)
    Y = torch.empty_like(X)
    ladj = torch.empty(N, device=dev, dtype=td)

    def layer_array(lays):
        dps = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p).T)).to(dev) for p in ps] for _, ps in lays]
        a = (lib.Layer * len(lays))()
        for i, ((op, ps), dp) in enumerate(zip(lays, dps)):
            a[i].op = op
            a[i].k = (np.asarray(ps[0]).shape[1] if np.asarray(ps[0]).ndim == 2 else 1) if op == 5 else 0
            for q, t in enumerate(dp):
                a[i].p[q] = t.data_ptr()
        return a, dps

    arr, dparams = layer_array(layers)
    dt0 = lib.ENF_F32 if args.dtype == "f32" else lib.ENF_F64
    if args.inverse:  # the inverse reads the forward's outputs (as bench.py --inverse)
        farr, fdp = layer_array(fwd)
        lib.check(L.enf_flow_apply(dt0, D, N, X.data_ptr(), D, Y.data_ptr(), D, ladj.data_ptr(), 0, farr, len(fwd), None))
        torch.cuda.synchronize()
        X, Y = Y, X
    st = torch.cuda.current_stream(dev)
    dt = lib.ENF_F32 if args.dtype == "f32" else lib.ENF_F64

    flush = torch.empty(args.flush_mb << 18, device=dev, dtype=torch.float32) if args.flush_mb else None

    def step():
        if flush is not None:
            flush.fill_(1.0)
        lib.check(L.enf_flow_apply(dt, D, N, X.data_ptr(), D, Y.data_ptr(), D, ladj.data_ptr(), 0, arr, len(layers),
                                   st.cuda_stream))

    import time

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.settle_ms:
        for _ in range(5):
            step()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.steps):
        step()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    esz = 4 if args.dtype == "f32" else 8
    knobs = {k: v for k, v in os.environ.items() if k.startswith("ENF_")}
    # bitwise fingerprint of the outputs (variants with identical arithmetic must agree exactly)
    import hashlib
    fp = hashlib.sha1(Y.cpu().numpy().tobytes() + ladj.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"tag": args.tag, "flush_mb": args.flush_mb, "lib": os.path.basename(lib.LIB_PATH), "knobs": knobs, "D": D, "N": N,
                      "pairs": args.pairs, "pattern": args.pattern, "dtype": args.dtype, "kernel_ms": ms, "out_sha1": fp,
                      "samples_per_s": N / (ms * 1e-3),
                      "hbm_frac": N * (2 * D + 1) * esz / (ms * 1e-3) / 8e12}))


if __name__ == "__main__":
    main()
