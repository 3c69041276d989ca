"""Config 5 benchmark: optimize_whitening training steps.

Data: X = f_true^{-1}(Z), Z ~ N(0,1) (D = 32, N = 1e7 columns, fp32), generated on the device with
the library's own inverse flow; trainable: a differently seeded J4∘H4∘…∘J1∘H1 flow; ADAGrad
(eta = 0.1); nbatches = 100 -> global minibatch B = 1e5. A step is one minibatch of
src/optimize_whitening.jl:37-41: the fused forward+backward negll gradient over this rank's share
(enf_flow_negll_grad), the cross-rank sum (torch.distributed all-reduce = RCCL; none at world 1),
ADAGrad on every trainable vector (enf_adagrad_step) and the Householder re-normalisation.

    python bench_train.py [--gpus N --steps 100 --warmup 5 --D 32 --N 10000000 --nbatches 100]

--gpus N > 1 started by hand launches its N ranks itself (enf_launch.py), one process per GPU. At
world > 1 the cross-rank sum is RCCL called through libenf (EnfComm, enf_allreduce_sum) on the
kernels' own stream, so the whole data-parallel step -- gradient, all-reduce, update -- is captured
into the HIP graph with the other timed steps (--graph 1, default). --selftest-cpu runs the rank
plumbing (launch, minibatch shares, a gloo sum of a stand-in gradient, max-over-ranks) on the CPU for
the tests; it measures nothing.

Prints one JSON line (rank 0): steps/s, samples/s (global minibatch samples per second), the
per-step time of the gradient kernel pair (HIP events), every rank's time and the negll trajectory
endpoints.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import enf_launch  # noqa: E402
from bench import build_flow, gather_ranks, max_over_ranks  # noqa: E402


def train_leg_selftest(world, rank, N=10_000_000, nbatches=100, steps=100):
    """The data-parallel step's plumbing on the CPU (torch.distributed already initialised on gloo when
    world > 1): each rank sums a stand-in gradient over its share of every minibatch, the shares are
    summed across ranks, and every rank must end with the same update. Returns the record (rank 0's is
    printed); measures nothing."""
    import torch

    from enf_pkg import load

    plan = load().minibatch_plan(N, nbatches, rank, world)
    Xh = np.cos(np.arange(N, dtype=np.float64))
    theta = torch.zeros(3, dtype=torch.float64)
    t0 = time.perf_counter()
    for i in range(steps):
        B, lo, hi = plan[i % len(plan)]
        g = torch.tensor([float(Xh[lo:hi].sum()), float((Xh[lo:hi] ** 2).sum()), float(hi - lo)], dtype=torch.float64)
        if world > 1:
            torch.distributed.all_reduce(g)
        assert g[2].item() == B  # the rank shares tile the minibatch exactly once
        theta -= 0.1 * g / B
    wall = time.perf_counter() - t0
    per_rank = gather_ranks(wall, torch.device("cpu"), world, rank)
    th = gather_ranks(float(theta.sum()), torch.device("cpu"), world, rank)
    return {"metric": "optimize_whitening training steps/s (config 5)", "value": steps / max(per_rank),
            "unit": "steps/s", "n_gpus": world, "steps": steps, "selftest": "cpu (measures nothing)",
            "per_rank_s": per_rank, "ranks_agree": len(set(th)) == 1,
            "step": step_description(world == 1, world, "enf", True),
            "config": {"parallelism": f"dp{world}", "B": plan[0][0]}}


def step_description(fused, world, comm_kind, graph, dp_fused=False):
    """What one timed config-5 step runs (the `step` / `launch` fields of the record)."""
    if fused:
        return "enf_whitening_step (fused, 1 rank)"
    if dp_fused:
        return ("enf_whitening_step_dp (gradient, RCCL sum of the slice totals over xGMI on the kernels' stream"
                + (", captured in the HIP graph" if graph else "") + ", one tail launch)")
    comm = ("libenf EnfComm (RCCL over xGMI on the kernels' stream" + (", captured in the HIP graph)" if graph else ")")
            if comm_kind == "enf" else "torch.distributed all_reduce (eager)")
    return f"enf_flow_negll_grad + {comm} + enf_whitening_apply"


def selftest_cpu(args, world, rank):
    """The harness on gloo without a GPU (train_leg_selftest)."""
    import torch

    if world > 1:
        torch.distributed.init_process_group("gloo")
    res = train_leg_selftest(world, rank, args.N, args.nbatches, args.steps)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--selftest-cpu", action="store_true", help="CPU tests only: rank plumbing on gloo")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--N", type=int, default=10_000_000, help="total samples (all ranks)")
    ap.add_argument("--nbatches", type=int, default=100)
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--history", default="", help="write the per-step negll to this file (JSON list)")
    ap.add_argument("--graph", type=int, default=1,
                    help="capture the timed steps (incl. the RCCL all-reduce at world > 1) once into a HIP graph "
                         "and replay it (0: eager launches)")
    ap.add_argument("--diag", action="store_true",
                    help="tools only: run on the diagnostics library (libenf_diag.so, ENF_* knobs) instead of libenf.so")
    ap.add_argument("--comm", default="enf", choices=["enf", "torch"],
                    help="world > 1: RCCL through libenf on the kernels' stream (enf; graph-capturable) or "
                         "torch.distributed.all_reduce (torch; eager only)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one process: rank 0's data-parallel step at this world size (its share of each minibatch)")
    ap.add_argument("--breakdown", action="store_true", help="per-phase event times of eager steps after the timed ones")
    ap.add_argument("--example", choices=["1d", "2d"], default=None,
                    help="the reference examples' training loops (examples/nf_example_1d.jl, nf_example_2d.jl): their "
                         "flows, N = 1e5, nbatches and nepochs, fp64; steps/s of graph-replayed epochs beside the "
                         "oracle's optimize_whitening on the host (one thread)")
    args = ap.parse_args()

    # N > 1 started by hand: start the N ranks as child processes before anything touches a GPU
    rc = enf_launch.spawn_ranks_if_needed(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world, rank, local_rank = enf_launch.rank_env()
    enf_launch.check_world(args.gpus, world)
    if args.selftest_cpu:
        return selftest_cpu(args, world, rank)
    import torch

    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.diag:
        from enf_pkg import load

        load()._lib.use_diagnostics_library()
    if args.example:
        print(json.dumps(example_leg(dev, args.example)))
        return
    res = train_leg(dev, world, rank, D=args.D, N=args.N, nbatches=args.nbatches, pairs=args.pairs, steps=args.steps,
                    warmup=args.warmup, graph=bool(args.graph), comm_kind=args.comm, history=args.history,
                    emulate_world=args.emulate_world or None, breakdown=args.breakdown)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


def train_leg(dev, world, rank, D=32, N=10_000_000, nbatches=100, pairs=4, steps=100, warmup=5, graph=True,
              comm_kind="enf", history="", emulate_world=None, breakdown=False, dp_fused=True):
    """Config 5 on this process's GPU as one rank of `world` (torch.distributed initialised by the
    caller when world > 1): returns the result record (the same on every rank; rank 0 prints it).
    Also run by bench.py after its headline measurement (`train` object of its JSON line).
    emulate_world=W (one process only): the data-parallel step of rank 0 of W ranks -- its share B/W of each
    minibatch, the gradient, a single-rank EnfComm all-reduce and enf_whitening_apply normalised by the whole
    minibatch B -- i.e. one rank's step at that world size without the cross-GPU transfer (the update differs
    from a real W-rank run, which sums every share; the timing is the rank's local work).
    breakdown=True: after the timed steps, `steps` eager steps with HIP events between the phases (gradient
    launches, all-reduce, update; or the fused call) -> their per-phase medians.
    dp_fused: the data-parallel step with an EnfComm as ONE call, enf_whitening_step_dp (gradient, RCCL sum of the
    double slice totals, one tail launch; round 4), else enf_flow_negll_grad + all-reduce + enf_whitening_apply."""
    import torch

    from enf_pkg import load

    enf = load()
    lib = enf._lib
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace, householder_batches, trainable_runs  # noqa: E402,E501

    mk = lambda layers: enf.compose(*[enf.HouseholderTrafo(ps[0]) if op == 5 else enf.JohnsonTrafo(*ps)
                                      for op, ps in reversed(layers)])
    # the data-generating flow's inverse (sinh layers) must stay finite over 4 layers: delta in [3, 5]
    ltrue = build_flow(D, pairs, np.float32, seed=7)
    rs = np.random.default_rng(7)
    for op, ps in ltrue:
        if op == 3:
            ps[1] = rs.uniform(3, 5, D).astype(np.float32)
    f_true = mk(ltrue)
    f0 = mk(build_flow(D, pairs, np.float32, seed=42))
    # every rank holds the whole sample set (columns are read by rank shares of each minibatch)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    Z = torch.randn((N, D), generator=g, device=dev, dtype=torch.float32).t()
    X = enf.inverse(f_true)(Z)
    del Z
    if emulate_world and world != 1:
        raise ValueError("emulate_world runs in a single process")
    plan = enf.minibatch_plan(N, nbatches, 0 if emulate_world else rank, emulate_world or world)
    state = FlowState(f0, D, torch.float32, dev, enf.ADAGrad())
    out = torch.zeros(1 + state.nparams, dtype=torch.float32, device=dev)
    ws = _workspace(state, max(B for B, _, _ in plan))
    segs = trainable_runs(state)
    hbatches = householder_batches(state)
    L = lib.lib()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ldx = X.stride(1)
    opt = enf.ADAGrad()
    hist = []

    fused = world == 1 and not emulate_world and os.environ.get("BENCH_UNFUSED", "0") != "1"
    comm = None
    if not fused and comm_kind == "enf":
        comm = enf.EnfComm.from_process_group() if world > 1 else enf.EnfComm.single()
    runs = np.ascontiguousarray(np.array(segs, dtype=np.int64).reshape(-1))
    hbs = np.ascontiguousarray(np.array(hbatches, dtype=np.int64).reshape(-1))
    hdev = torch.zeros(warmup + steps, dtype=torch.float64, device=dev)

    def step(i, ev=None, sh=sh, ph=None):
        # ev: events around the gradient launches (the timed eager steps); ph: [e0, e1, e2, e3] around the
        # gradient, the all-reduce and the update (breakdown)
        B, lo, hi = plan[i % len(plan)]
        if ph is not None:
            ph[0].record(stream)
        if fused:  # enf_whitening_step: gradient, loss, ADAGrad, re-normalisation (2 launches; 1 for one-block batches)
            if ev is not None:
                ev[0].record(stream)
            lib.check(L.enf_whitening_step(lib.ENF_F32, D, hi - lo, X[:, lo:hi].data_ptr(), ldx, state.layers(),
                                           len(state.trafos), state.theta.data_ptr(), state.acc.data_ptr(),
                                           runs.ctypes.data, len(segs), hbs.ctypes.data, len(hbatches), opt.eta,
                                           opt.epsilon, hdev[i:].data_ptr(), ws.data_ptr(), ws.numel() * 8, sh))
            if ev is not None:
                ev[1].record(stream)
            if ph is not None:
                ph[3].record(stream)
            return hdev[i:i + 1]
        if dp_fused and comm is not None:  # enf_whitening_step_dp: gradient, RCCL sum, tail
            if ev is not None:
                ev[0].record(stream)
            lib.check(L.enf_whitening_step_dp(lib.ENF_F32, D, hi - lo, X[:, lo:hi].data_ptr(), ldx, state.layers(),
                                              len(state.trafos), state.theta.data_ptr(), state.acc.data_ptr(),
                                              runs.ctypes.data, len(segs), hbs.ctypes.data, len(hbatches), opt.eta,
                                              opt.epsilon, B, hdev[i:].data_ptr(), comm.handle, ws.data_ptr(),
                                              ws.numel() * 8, sh))
            if ev is not None:
                ev[1].record(stream)
            if ph is not None:
                ph[3].record(stream)
            return hdev[i:i + 1]
        out.zero_()
        if ev is not None:
            ev[0].record(stream)
        if hi > lo:
            lib.check(L.enf_flow_negll_grad(lib.ENF_F32, D, hi - lo, X[:, lo:hi].data_ptr(), ldx, state.layers(),
                                            len(state.trafos), out.data_ptr(), ws.data_ptr(), ws.numel() * 8, sh))
        if ev is not None:
            ev[1].record(stream)
        if ph is not None:
            ph[1].record(stream)
        if comm is not None:
            comm.allreduce_sum_(out, sh)  # RCCL on the kernels' stream
        else:
            enf.allreduce_sum_(out, world)
        if ph is not None:
            ph[2].record(stream)
        # loss, ADAGrad and re-normalisation on every rank in one launch
        lib.check(L.enf_whitening_apply(lib.ENF_F32, D, state.nparams, out.data_ptr(), B, state.theta.data_ptr(),
                                        state.acc.data_ptr(), runs.ctypes.data, len(segs), hbs.ctypes.data,
                                        len(hbatches), opt.eta, opt.epsilon, hdev[i:].data_ptr(), sh))
        if ph is not None:
            ph[3].record(stream)
        return hdev[i:i + 1]

    for i in range(warmup):
        hist.append(step(i))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    graph = graph and (fused or comm is not None)
    if graph:
        # the timed steps as one HIP graph: captured (nothing runs), replayed once untimed (this
        # advances the optimizer by steps more steps), then replayed once timed
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            cs = torch.cuda.current_stream().cuda_stream
            for i in range(steps):
                step(warmup + i, None, cs)
        cg.replay()
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    if graph:
        evs = evs[:1]
        evs[0][0].record(stream)
        cg.replay()
        evs[0][1].record(stream)
        hist.append(hdev[warmup:warmup + steps])
    else:
        for i in range(steps):
            hist.append(step(warmup + i, evs[i]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    grad_ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
    if graph:
        grad_ms /= steps  # the replay's event pair brackets all steps
    per_rank_ms = gather_ranks(wall / steps * 1e3, dev, world, rank)
    wall, grad_ms_max = max_over_ranks([wall, grad_ms], dev, world)
    samples = sum(plan[(warmup + i) % len(plan)][0] for i in range(steps))
    hist_vals = torch.cat(hist).cpu()  # (before the breakdown's steps overwrite the device history)
    phases = None
    if breakdown:
        # eager steps with events between the phases (after the timed region; advances the optimizer further)
        evp = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
        for i in range(steps):
            step(warmup + i, None, sh, evp[i])
        torch.cuda.synchronize()
        med = lambda xs: float(np.median(xs))
        if fused or (dp_fused and comm is not None):
            phases = {"fused_step_ms": med([e[0].elapsed_time(e[3]) for e in evp]),
                      "launches": "enf_whitening_step: gradient kernel + one reduction/update launch (a batch that fits "
                                              "one block: a single fused launch)" if fused else
                                  "enf_whitening_step_dp: gradient kernel + block-partial sum + RCCL all-reduce of "
                                  "1 + nparams doubles + update"}
        else:
            phases = {"gradient_ms": med([e[0].elapsed_time(e[1]) for e in evp]),
                      "allreduce_ms": med([e[1].elapsed_time(e[2]) for e in evp]),
                      "update_ms": med([e[2].elapsed_time(e[3]) for e in evp]),
                      "step_ms": med([e[0].elapsed_time(e[3]) for e in evp]),
                      "launches": "gradient: out.zero_ + gradient kernel + one reduction launch; all-reduce: RCCL; "
                                  "update: enf_whitening_apply (1 launch)"}
        phases["mode"] = "eager, HIP events between the phases (median over the steps)"
    negll = [float(h) for h in hist_vals]
    if history and rank == 0:
        with open(history, "w") as f:
            json.dump(negll, f)
    res = {
        "metric": "optimize_whitening training steps/s (config 5)",
        "value": steps / wall, "unit": "steps/s", "samples_per_s": samples / wall,
        "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": wall / steps * 1e3,
        "grad_kernel_ms_median" if not fused else "fused_step_ms_median": grad_ms,
        "grad_kernel_ms_max_rank" if not fused else "fused_step_ms_max_rank": grad_ms_max, "dtype": "f32",
        "launch": "HIP graph of the timed steps (torch.cuda.CUDAGraph), replayed" if graph else "eager",
        "step": step_description(fused, world, "enf" if comm is not None else "torch", graph,
                                 dp_fused and comm is not None),
        "per_rank_ms_per_step": per_rank_ms,
        "data": "synthetic: X = f_true^-1(Z), Z ~ N(0,1) (torch Philox 0x5EED), f_true seed 7, init seed 42",
        "config": {"workload": f"optimize_whitening D={D}, N={N}, nbatches={nbatches} "
                               f"(B={plan[0][0]}), {pairs}x(J∘H), ADAGrad(0.1)",
                   "per_rank_share": plan[0][2] - plan[0][1], "parallelism": f"dp{world}",
                   "emulated_world": emulate_world},
        "phases": phases,
        "negll_first": negll[0], "negll_last": negll[-1],
    }
    if graph:
        # the graph holds the captured RCCL all-reduce: release it (and let its work drain) before the
        # communicator (the order optimize_whitening uses)
        del cg
        torch.cuda.synchronize()
    if comm is not None:
        comm.close()
    return res


def example_flows(example):
    """(D, true flow, initial flow, nbatches, nepochs) of a reference example, layers innermost first:
    nf_example_1d.jl:8-10,20-29 (X = CenterStretch o JohnsonTrafo (randn), initial J o inverse(C) o J o inverse(C),
    nbatches 100, nepochs 10) and nf_example_2d.jl:12-15,21-30 (X = ScaleShift o Householder o CenterStretch
    (randn), initial inverse(C) o inverse(H(randn(2))) o ScaleShift, nbatches 1000, nepochs 10)."""
    a = lambda *v: np.array(v, dtype=np.float64)
    if example == "1d":
        true = [(3, [a(10.0), a(3.5), a(10.0), a(1.0)]), (1, [a(4.0), a(1.0), a(0.0)])]
        init = [(2, [a(0.0), a(1.0), a(0.0)]), (3, [a(0.0), a(5.0), a(0.0), a(5.0)]),
                (2, [a(0.0), a(1.0), a(0.0)]), (3, [a(0.0), a(5.0), a(0.0), a(5.0)])]
        return 1, true, init, 100, 10
    rs = np.random.default_rng(2)
    true = [(1, [a(4.0, 4.1), a(2.0, 2.1), a(3.0, 3.1)]), (5, [a(1.0, 0.3)]), (0, [a(1.3, 0.4), a(2.5, -1.2)])]
    init = [(0, [a(1.0, 1.0), a(0.0, 0.0)]), (5, [rs.standard_normal(2)]), (2, [a(0.0, 0.0), a(1.0, 1.0), a(0.0, 0.0)])]
    return 2, true, init, 1000, 10


def example_leg(dev, example, N=100_000):
    """The reference example's optimize_whitening on the device (fp64, ADAGrad, graph=True: one epoch captured as
    a HIP graph and replayed per epoch) after one untimed warm-up run; steps/s over the replayed epochs (the
    capture of the epoch's launches is timed separately), beside the oracle's optimize_whitening on the host."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # bench: the CPU baseline and the parity check of the history only

    from enf_pkg import load

    enf = load()
    D, true, init, nbatches, nepochs = example_flows(example)
    rng = np.random.default_rng(1)
    XW = np.asfortranarray(rng.standard_normal((D, N)))
    X, _ = oracle.flow_apply(true, XW)
    X = np.asfortranarray(X)
    mk = lambda layers: enf.compose(*[
        {0: lambda ps: enf.ScaleShiftTrafo(*ps), 1: lambda ps: enf.CenterStretch(*ps),
         2: lambda ps: enf.CenterContract(*ps), 3: lambda ps: enf.JohnsonTrafo(*ps),
         5: lambda ps: enf.HouseholderTrafo(ps[0])}[op](ps) for op, ps in reversed(layers)])
    Xd = torch.from_numpy(np.ascontiguousarray(X.T)).to(dev).t()
    opt = enf.ADAGrad()
    enf.optimize_whitening(Xd, mk(init), opt, nbatches=nbatches, nepochs=1, graph=True)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = enf.optimize_whitening(Xd, mk(init), opt, nbatches=nbatches, nepochs=nepochs, graph=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # the replay rate alone: the same epoch graph replayed (capture excluded)
    from euclidiannormalizingflows_jl_amd.train import FlowState, _workspace, householder_batches, trainable_runs

    lib = enf._lib
    L = lib.lib()
    state = FlowState(mk(init), D, torch.float64, dev, opt)
    plan = enf.minibatch_plan(N, nbatches, 0, 1)
    ws = _workspace(state, max(B for B, _, _ in plan))
    runs = np.ascontiguousarray(np.array(trainable_runs(state), dtype=np.int64).reshape(-1))
    hbs = np.ascontiguousarray(np.array(householder_batches(state), dtype=np.int64).reshape(-1))
    hep = torch.zeros(len(plan), dtype=torch.float64, device=dev)
    cg = torch.cuda.CUDAGraph()
    tc = time.perf_counter()
    with torch.cuda.graph(cg):
        st = torch.cuda.current_stream().cuda_stream
        # the epoch as optimize_whitening runs it on one rank: one enf_whitening_epoch call (round 5: a single launch
        # whose one block walks the minibatches)
        lib.check(L.enf_whitening_epoch(lib.ENF_F64 | lib.ENF_NEGLL_ZYGOTE, D, N, Xd.data_ptr(), D, plan[0][0],
                                        state.layers(),
                                        len(state.trafos), state.theta.data_ptr(), state.acc.data_ptr(),
                                        runs.ctypes.data, len(runs) // 2, hbs.ctypes.data, len(hbs) // 3, opt.eta,
                                        opt.epsilon, hep.data_ptr(), ws.data_ptr(), ws.numel() * 8, st))
    capture_s = time.perf_counter() - tc
    cg.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream()
    e0.record(stream)
    for _ in range(nepochs):
        cg.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    replay_ms = e0.elapsed_time(e1)
    del cg
    steps = nepochs * len(plan)
    # the oracle on the host, one thread: the same loop (gradient on the CPU, ADAGrad, normalize!)
    tcpu = time.perf_counter()
    # (zygote=True: the history the reference records, its ScaleShift ladj missing under Zygote, as the drop-in's default)
    _, _, hist_ref = oracle.optimize_whitening(init, X, nbatches=nbatches, nepochs=nepochs, eta=opt.eta,
                                               epsilon=opt.epsilon, zygote=True)
    cpu_s = time.perf_counter() - tcpu
    hist = np.asarray(r.negll_history)
    B = plan[0][0]
    return {"metric": f"optimize_whitening training steps/s (reference example {example})", "unit": "steps/s",
            "value": steps / (replay_ms * 1e-3), "us_per_step": replay_ms * 1e3 / steps,
            "launch": "one epoch (one enf_whitening_epoch call) captured as a HIP graph, replayed nepochs times "
                      "(capture excluded)",
            "end_to_end": {"steps_per_s": steps / wall, "wall_s": wall,
                           "what": "optimize_whitening(graph=True) call: capture + replays + history copy"},
            "capture_s": capture_s, "steps": steps, "dtype": "f64",
            "config": {"workload": f"examples/nf_example_{example}.jl: D={D}, N={N}, nbatches={nbatches} (B={B}), "
                                   f"nepochs={nepochs}, {'JKJK' if example == '1d' else 'KHS'} initial flow, ADAGrad",
                       "flow_letters_application_order": "KJKJ" if example == "1d" else "SHK"},
            "cpu_baseline": {"value": steps / cpu_s, "unit": "steps/s", "cores": 1, "kind": "port",
                             "sample": f"the whole loop ({steps} steps) in the oracle (oracle/enf_oracle_grad.c "
                                       f"or_optimize_whitening_f64: the reference-structured reverse pass), one thread",
                             "seconds": cpu_s},
            "parity": {"history_max_rel_diff_vs_oracle": float(np.max(np.abs(hist - hist_ref) / np.abs(hist_ref))),
                       "history": "as the reference records it under Zygote (similar_fill quirk: a ScaleShiftTrafo's "
                                  "ladj primal is zero, src/abstract_trafo.jl:30-33), device and oracle alike",
                       "negll_first": float(hist[0]), "negll_last": float(hist[-1])},
            "data": "synthetic: X = the example's true flow of randn (numpy seed 1), as the example script"}


if __name__ == "__main__":
    main()
