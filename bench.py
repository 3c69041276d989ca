"""Headline benchmark: samples/s of forward + log|det J| through the composed flow
(BASELINE.json metric; SURVEY.md §8(d) config 3: J4∘H4∘J3∘H3∘J2∘H2∘J1∘H1, D=32, N=1e7 per GPU, fp32).

A "step" is one enf_flow_apply over the whole N-sample batch (one fused launch): X is read once,
Y (D x N) and ladj (N) are written once, inputs already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W] [--D 32 --N 10000000 --pairs 4 --dtype f32]

Multi-GPU (one process per GPU, launched by torch.distributed.run): every rank processes its own
N-sample shard of the batch (columns are independent, no data-path collective) -> weak scaling;
the timed region is bracketed by barriers + device syncs and the max over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
MFMA_NOTE = "elementwise/rank-1 maps: HBM roofline (SURVEY.md §8(d))"


def build_flow(D, pairs, np_dtype, seed=42, pattern=None):
    """Parameters from a host RNG with seed 42 in per-layer order.
    pattern: layer letters applied in order (H = Householder, J = Johnson); default "HJ" * pairs."""
    rng = np.random.default_rng(seed)
    layers = []
    for ch in (pattern or "HJ" * pairs):
        if ch == "H":
            layers.append((5, [rng.standard_normal(D).astype(np_dtype)]))
        elif ch == "J":
            layers.append((3, [rng.uniform(-1, 1, D).astype(np_dtype), rng.uniform(0.5, 2, D).astype(np_dtype),
                               rng.uniform(-0.5, 0.5, D).astype(np_dtype), rng.uniform(0.5, 2, D).astype(np_dtype)]))
        else:
            raise ValueError(f"unknown layer letter {ch!r}")
    return layers


def pmc_evidence(D, N, args, kern_ms):
    """HBM traffic per launch and the VALU issue picture of the same kernel on the same workload,
    from the committed rocprofv3 PMC passes (profiles/r01_pmc_traffic.json, tools/pmc.sh): traffic =
    FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE; VALU issue cycles per SIMD = (4 x plain +
    8 x transcendental wave64 instructions) / 1024 SIMDs (MI355X_MICROARCH.md issue costs)."""
    prof = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")
    try:
        with open(prof) as f:
            tr = json.load(f)
    except (OSError, ValueError):
        return None, None
    if not (tr.get("D") == D and tr.get("N") == N and tr.get("dtype") == args.dtype and tr.get("pairs") == args.pairs
            and args.pattern is None):
        return None, None
    c = tr.get("counters", {})
    valu = None
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_VALU_TRANS_F32" in c:
        trans = c["SQ_INSTS_VALU_TRANS_F32"]
        cyc = (4.0 * (c["SQ_INSTS_VALU"] - trans) + 8.0 * trans) / 1024.0
        clk = tr.get("effective_clock_ghz")
        valu = {"insts_per_launch": c["SQ_INSTS_VALU"], "trans_insts_per_launch": trans,
                "issue_cycles_per_simd": cyc, "pmc_effective_clock_ghz": clk,
                "pmc_kernel_ms": tr.get("median_duration_ns_profiled", 0) / 1e6,
                "issue_frac_in_pmc_run": (cyc / (clk * 1e9 * tr["median_duration_ns_profiled"] * 1e-9)
                                          if clk and tr.get("median_duration_ns_profiled") else None),
                "source": "profiles/r01_pmc_traffic.json"}
    return tr.get("hbm_bytes_per_launch"), valu


def max_over_ranks(values, device, world):
    """Element-wise max over ranks of per-rank values (the timed region's wall time and kernel
    time): the whole job is as slow as its slowest GPU. torch.distributed all-reduce(MAX)
    (RCCL between GPUs; gloo in the CPU tests)."""
    t = torch.tensor(values, device=device, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return [float(v) for v in t]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--N", type=int, default=10_000_000, help="samples per GPU")
    ap.add_argument("--pairs", type=int, default=4, help="number of (Householder, Johnson) pairs")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-samples", type=int, default=3_000_000)
    ap.add_argument("--pattern", default=None, help="diagnostic layer pattern, e.g. HHHHHHHH (overrides --pairs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from enf_pkg import load

    enf = load()
    lib = enf._lib
    np_dtype = np.float32 if args.dtype == "f32" else np.float64
    t_dtype = torch.float32 if args.dtype == "f32" else torch.float64
    esz = 4 if args.dtype == "f32" else 8
    D, N = args.D, args.N
    layers = build_flow(D, args.pairs, np_dtype, pattern=args.pattern)

    # synthetic X: N(0,1) columns from torch's counter-based (Philox) CUDA generator; each rank
    # draws its own shard (global column offset = rank * N)
    g = torch.Generator(device=dev).manual_seed(0x5EED + rank)
    X = torch.randn((N, D), generator=g, device=dev, dtype=t_dtype)  # row-major N x D == column-major D x N
    Y = torch.empty_like(X)
    ladj = torch.empty(N, device=dev, dtype=t_dtype)
    dparams = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p))).to(dev) for p in ps] for _, ps in layers]
    arr = (lib.Layer * len(layers))()
    for i, ((op, ps), dp) in enumerate(zip(layers, dparams)):
        arr[i].op, arr[i].k = op, 1 if op == 5 else 0
        for q, t in enumerate(dp):
            arr[i].p[q] = t.data_ptr()
    L = lib.lib()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    dt_code = lib.ENF_F32 if args.dtype == "f32" else lib.ENF_F64

    def step():
        lib.check(L.enf_flow_apply(dt_code, D, N, X.data_ptr(), D, Y.data_ptr(), D, ladj.data_ptr(), 0,
                                   arr, len(layers), sh))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the launch stream
    t_local, kern_ms_max = max_over_ranks([wall, kern_ms], dev, world)
    ms_per_step = t_local / args.steps * 1e3
    total_samples = N * world * args.steps
    value = total_samples / t_local

    bytes_per_launch = N * (2 * D + 1) * esz  # read X, write Y, write ladj
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic, valu = pmc_evidence(D, N, args, kern_ms)
    copy_gbs = copy_ceiling(X, Y, stream)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(layers, D, np_dtype, args.cpu_samples)

    if rank == 0:
        out = {
            "metric": "samples/sec fwd+logdetjac through composed flow, D=32 N=1e7, at 1/2/4/8 GPUs",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic: X ~ N(0,1) (torch Philox, seed 0x5EED+rank); params seed 42",
            "config": {"workload": f"{'∘'.join(reversed(args.pattern or 'HJ' * args.pairs))} composed flow "
                                   f"fwd+ladj, D={D}, N={N} per GPU",
                       "D": D, "N_per_gpu": N, "layers": len(layers), "parallelism": f"sample-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_ms": kern_ms, "kernel_ms_max_rank": kern_ms_max,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "torch_copy_GBps": copy_gbs, "frac_of_torch_copy": achieved / copy_gbs},
            "valu": valu,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


def copy_ceiling(X, Y, stream, reps=10):
    """Practical streaming ceiling of this GPU for the same bytes (confirm the HBM
    peak with a copy): torch's device copy of X into Y (N*D values read and written), timed with HIP
    events on the launch stream. Y is overwritten (after the timed steps)."""
    Y.copy_(X)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        Y.copy_(X)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2 * X.numel() * X.element_size() / (ms * 1e-3) / 1e9


def cpu_baseline(layers, D, np_dtype, nsamp):
    """The oracle (CPU restatement of the reference algorithm; Julia is unavailable) timed on a bounded
    sample of the same workload on this host: reference-structured, 1 thread (layer by layer,
    materialising Y and the D x N ladj temporaries as the Julia broadcasts do)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # bench cpu_baseline leg only

    oracle.build()
    rng = np.random.default_rng(1)
    X = np.asfortranarray(rng.standard_normal((D, nsamp)).astype(np_dtype))
    t0 = time.perf_counter()
    oracle.flow_apply(layers, X)
    t1 = time.perf_counter() - t0
    nthr = min(os.cpu_count() or 1, 16)
    t0 = time.perf_counter()
    oracle.flow_apply(layers, X, nthreads=nthr)
    tm = time.perf_counter() - t0
    return {"value": nsamp / t1, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{nsamp} samples of the same flow (D={D}), reference-structured C restatement, 1 thread, "
                      f"{t1:.1f} s",
            "openmp": {"value": nsamp / tm, "cores": nthr, "seconds": tm}}


if __name__ == "__main__":
    main()
