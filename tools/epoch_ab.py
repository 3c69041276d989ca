"""A/B of one reference example's epoch launch (design tool, not product): the epoch of bench_train.py's example
leg (one enf_whitening_epoch call captured as a HIP graph, replayed) with and without ENF_NEGLL_ZYGOTE, on the
library at --lib (default: the product's). One JSON line per configuration.
python tools/epoch_ab.py --example 2d [--lib tools/ab/libenf_r5.so] [--no-zygote-only] --tag NAME
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--example", choices=["1d", "2d"], default="2d")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--no-zygote-only", action="store_true", help="a library without the flag (before round 6)")
    ap.add_argument("--tag", default="")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    import oracle
    from bench_train import example_flows
    from enf_pkg import load

    enf = load()
    if args.lib:
        enf._lib.use_diagnostics_library(os.path.join(ROOT, args.lib))
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace, householder_batches, trainable_runs

    dev = torch.device("cuda:0")
    D, true, init, nbatches, _ = example_flows(args.example)
    N = 100_000
    rng = np.random.default_rng(1)
    X, _ = oracle.flow_apply(true, np.asfortranarray(rng.standard_normal((D, N))))
    Xd = torch.from_numpy(np.ascontiguousarray(np.asfortranarray(X).T)).to(dev).t()
    mk = lambda layers: enf.compose(*[
        {0: lambda ps: enf.ScaleShiftTrafo(*ps), 1: lambda ps: enf.CenterStretch(*ps),
         2: lambda ps: enf.CenterContract(*ps), 3: lambda ps: enf.JohnsonTrafo(*ps),
         5: lambda ps: enf.HouseholderTrafo(ps[0])}[op](ps) for op, ps in reversed(layers)])
    lib = enf._lib
    L = lib.lib()
    opt = enf.ADAGrad()
    plan = enf.minibatch_plan(N, nbatches, 0, 1)
    flags = [0] if args.no_zygote_only else [0, lib.ENF_NEGLL_ZYGOTE, 0, lib.ENF_NEGLL_ZYGOTE]
    for fl in flags:
        state = FlowState(mk(init), D, torch.float64, dev, opt)
        ws = _workspace(state, max(B for B, _, _ in plan))
        runs = np.ascontiguousarray(np.array(trainable_runs(state), dtype=np.int64).reshape(-1))
        hbs = np.ascontiguousarray(np.array(householder_batches(state), dtype=np.int64).reshape(-1))
        hep = torch.zeros(len(plan), dtype=torch.float64, device=dev)
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            st = torch.cuda.current_stream().cuda_stream
            lib.check(L.enf_whitening_epoch(lib.ENF_F64 | fl, D, N, Xd.data_ptr(), D, plan[0][0], state.layers(),
                                            len(state.trafos), state.theta.data_ptr(), state.acc.data_ptr(),
                                            runs.ctypes.data, len(runs) // 2, hbs.ctypes.data, len(hbs) // 3,
                                            opt.eta, opt.epsilon, hep.data_ptr(), ws.data_ptr(), ws.numel() * 8, st))
        cg.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            cg.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (args.reps * len(plan))
        print(json.dumps({"tag": args.tag, "example": args.example, "lib": args.lib or "libenf.so",
                          "zygote": bool(fl), "us_per_step": us}), flush=True)
        del cg


if __name__ == "__main__":
    main()
