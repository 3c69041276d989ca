"""Headline benchmark: samples/s of forward + log|det J| through the composed flow
(BASELINE.json metric; SURVEY.md §8(d) config 3: J4∘H4∘J3∘H3∘J2∘H2∘J1∘H1, D=32, N=1e7 per GPU, fp32).

A "step" is one enf_flow_apply over the whole N-sample batch (one fused launch): X is read once,
Y (D x N) and ladj (N) are written once, inputs already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W] [--D 32 --N 10000000 --pairs 4 --dtype f32]

Multi-GPU: one process per GPU. Under torch.distributed.run (WORLD_SIZE set) each process is one
rank; `python bench.py --gpus N` started by hand starts the N ranks itself (enf_launch.py: child
processes under torch.distributed.run, before anything touches a GPU). Every rank processes its own
N-sample shard of the batch (columns are independent, src/abstract_trafo.jl:9: no data-path
collective) -> weak scaling; the timed region is bracketed by barriers + device syncs, value = all
ranks' samples / the max over ranks of the timed wall time, and the per-rank kernel times are
printed. `--selftest-cpu` runs the same harness (launch, barriers, max-over-ranks, aggregation) on
gloo with a CPU stand-in step, for the CPU tests; it measures nothing.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import enf_launch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md)
MFMA_NOTE = "elementwise/rank-1 maps: HBM roofline (SURVEY.md §8(d))"


LETTERS = {"S": 0, "C": 1, "K": 2, "J": 3, "I": 4, "H": 5}


def parse_pattern(pattern):
    """Layer letters in application order (innermost first): S = ScaleShiftTrafo, C = CenterStretch,
    K = CenterContract, J = JohnsonTrafo, I = JohnsonTrafoInv, H = one Householder reflection, H<k> = a
    chained HouseholderTrafo of k reflections (e.g. "H4JH4J"). Returns [(op, k)]."""
    import re

    out, pos = [], 0
    for m in re.finditer(r"([SCKJIH])(\d*)", pattern):
        if m.start() != pos:
            raise ValueError(f"unknown layer letter in pattern {pattern!r} at {pos}")
        k = int(m.group(2)) if m.group(2) else 1
        if m.group(2) and m.group(1) != "H":
            raise ValueError(f"only H takes a column count ({m.group(0)!r})")
        out.append((LETTERS[m.group(1)], k))
        pos = m.end()
    if pos != len(pattern) or not out:
        raise ValueError(f"bad pattern {pattern!r}")
    return out


def build_flow(D, pairs, np_dtype, seed=42, pattern=None):
    """Parameters from a host RNG with seed 42 in per-layer order (the Center and ScaleShift
    distributions of tests/parity.py rand_params). pattern: see parse_pattern; default "HJ" * pairs."""
    rng = np.random.default_rng(seed)
    u = lambda lo, hi: rng.uniform(lo, hi, D).astype(np_dtype)
    layers = []
    for op, k in parse_pattern(pattern or "HJ" * pairs):
        if op == 5:
            V = rng.standard_normal((D, k)).astype(np_dtype)
            layers.append((5, [V[:, 0] if k == 1 else np.asfortranarray(V)]))
        elif op in (3, 4):
            layers.append((op, [u(-1, 1), u(0.5, 2), u(-0.5, 0.5), u(0.5, 2)]))
        elif op in (1, 2):
            layers.append((op, [u(0, 2), u(0.5, 2), u(-0.5, 0.5)]))
        else:
            layers.append((0, [(np.where(rng.random(D) < 0.5, -1, 1) * rng.uniform(0.5, 2, D)).astype(np_dtype),
                               rng.standard_normal(D).astype(np_dtype)]))
    return layers


def invert_layers(layers):
    """Layers (innermost first) of inverse(f_n o ... o f_1): reversed order, each layer inverted as the
    reference's InverseFunctions.inverse methods do (scale_shift_trafo.jl:26-30: ScaleShift(1/a, -b/a);
    center_stretch.jl:45,69: CenterStretch <-> CenterContract; johnson_trafo.jl:82,107: JohnsonTrafo <->
    JohnsonTrafoInv; householder_trafo.jl:153-154: the reflection columns in reverse order)."""
    out = []
    for op, ps in reversed(layers):
        if op == 0:
            ai = (1 / ps[0]).astype(ps[0].dtype)
            out.append((0, [ai, (-ai * ps[1]).astype(ps[1].dtype)]))
        elif op in (1, 2):
            out.append((3 - op, ps))
        elif op in (3, 4):
            out.append((7 - op, ps))
        else:
            V = np.asarray(ps[0])
            out.append((5, [V if V.ndim == 1 else np.asfortranarray(V[:, ::-1])]))
    return out


def layer_letters(layers):
    inv = {v: k for k, v in LETTERS.items()}
    return "".join(inv[op] + (str(np.asarray(ps[0]).shape[1]) if op == 5 and np.asarray(ps[0]).ndim == 2 else "")
                   for op, ps in layers)


# Issue costs of gfx950 VALU wave-instructions at 4 waves per SIMD, measured on MI355X
# (tools/microbench5-8, profiles/r02_microbench_issue_costs.txt), in cycles at the microbenchmarks'
# clock: full-rate f32 fma/mul/add/sub and bit ops 2, half-rate ops (v_cmp, v_cndmask, v_bfi, DPP,
# v_max/min, any SGPR source or three source VGPRs in one bank) 4, transcendentals 7.5 (3.4 vs 1.0 ns)
ISSUE_CYC_FAST, ISSUE_CYC_TRANS = 2.0, 7.5
ISSUE_CYC_MIX_FAST, ISSUE_CYC_MIX_TRANS = 2.35, 12.1  # inside an FMA + transcendental mix (microbench21, round 3)


def pmc_evidence(D, N, args):
    """HBM traffic per launch and the VALU issue picture of the same kernel on the same workload from
    the newest committed rocprofv3 PMC summary (tools/pmc.sh + tools/pmc_summary.py; collected by
    separate `rocprofv3 --pmc` passes of `bench.py --no-cpu`, NOT in this run -- labelled as such):
    traffic = FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md §HBM) + WRITE_SIZE; issue-cycle
    floor per SIMD = (2 x non-transcendental + 7.5 x transcendental wave64 VALU instructions) / 1024
    SIMDs (a lower bound: half-rate instructions cost 4), against the cycles of the profiled launch
    (GRBM_GUI_ACTIVE clock x duration); SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES is the fraction of wave time
    spent waiting to issue (shared SIMD or dependency), SQ_INSTS_LDS the LDS instructions per launch."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_bench.json")))
    for prof in reversed(files):
        try:
            with open(prof) as f:
                tr = json.load(f)
        except (OSError, ValueError):
            continue
        if not (tr.get("D") == D and tr.get("N") == N and tr.get("dtype") == args.dtype
                and tr.get("pairs") == args.pairs and args.pattern is None):
            continue
        c = tr.get("counters", {})
        rel = os.path.relpath(prof, ROOT)
        traffic = {"bytes_per_launch": tr.get("hbm_bytes_per_launch"), "source": f"{rel} (rocprofv3 PMC passes, not this run)",
                   "kernel_git": tr.get("git")}
        valu = None
        if "SQ_INSTS_VALU" in c and "SQ_INSTS_VALU_TRANS_F32" in c:
            trans = c["SQ_INSTS_VALU_TRANS_F32"]
            cyc = (ISSUE_CYC_FAST * (c["SQ_INSTS_VALU"] - trans) + ISSUE_CYC_TRANS * trans) / 1024.0
            clk, dur = tr.get("effective_clock_ghz"), tr.get("median_duration_ns_profiled")
            # the same instructions priced at what they cost inside the loop's mix (round 3,
            # tools/microbench21: ~2.35 cycles per full-rate and ~12.1 per transcendental instruction when the
            # two interleave): the fraction of the launch's cycles that this instruction stream explains
            mix = (ISSUE_CYC_MIX_FAST * (c["SQ_INSTS_VALU"] - trans) + ISSUE_CYC_MIX_TRANS * trans) / 1024.0
            valu = {"insts_per_launch": c["SQ_INSTS_VALU"], "trans_insts_per_launch": trans,
                    "insts_per_element_pair": c["SQ_INSTS_VALU"] / (N * D * args.pairs / 64.0),
                    "issue_cycle_floor_per_simd": cyc, "pmc_effective_clock_ghz": clk,
                    "pmc_kernel_ms": dur / 1e6 if dur else None,
                    "issue_floor_frac": cyc / (clk * dur) if clk and dur else None,
                    "mix_cost_frac": mix / (clk * dur) if clk and dur else None,
                    "wait_inst_any_frac": tr.get("SQ_WAIT_INST_ANY_frac"),
                    "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
                    "source": f"{rel} (not this run)"}
        return traffic, valu
    return None, None


PMC_PASSES = ("FETCH_SIZE SQ_WAVES", "WRITE_SIZE",
              "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE",
              "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS")
KERNEL_PAT = "flow_hj_kernel"  # the headline kernel; --inverse: flow_hji_kernel, fp64: flow_hj64_kernel
# fp64 program (--dtype f64): one more pass with its instruction classes (wave64 VALU instructions)
PMC_PASS_F64 = ("SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 "
                "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64")
# fp64 issue costs on gfx950 at 2 waves per SIMD (profiles/r02_microbench15_fp64_costs.txt: fma/add/mul_f64
# 2.10 ns vs fma_f32 1.01 ns per wave-instruction, rcp/rsq_f64 6.84 ns), in cycles
ISSUE_CYC_F64, ISSUE_CYC_F64_TRANS = 4.2, 13.6


def kernel_pat(args):
    f64 = getattr(args, "dtype", "f32") == "f64"
    if getattr(args, "inverse", False):
        return "flow_hj64_kernel" if f64 else "flow_hji_kernel"
    return "flow_hj64_kernel" if f64 else KERNEL_PAT


def kernel_match(args, name):
    """True for the measured kernel's rocprofv3 name. The fp64 forward and inverse programs are one template,
    flow_hj64_kernel<D, U, LM, PAD, OCC, INV> (round 4): its last argument tells them apart (the inverse leg's
    untimed forward pass runs the forward one)."""
    if kernel_pat(args) not in name:
        return False
    m = re.search(r"flow_hj64_kernel<[^>]*, (true|false)>", name)
    return m is None or (m.group(1) == "true") == bool(getattr(args, "inverse", False))
PMC_BUDGET_S = 180.0  # all in-run profiler passes together (bench.py's default run stays within minutes)


def _run_group(cmd, timeout_s, log):
    """Run cmd in its own process group; on timeout kill the whole group (rocprofv3 and the program it
    runs). Returns the exit status (None on timeout)."""
    import signal
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "TORCHELASTIC_RUN_ID")}
    with open(log, "w") as lf:
        p = subprocess.Popen(cmd, stdout=lf, stderr=subprocess.STDOUT, start_new_session=True, cwd=ROOT, env=env)
        try:
            return p.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return None


def pmc_live(D, N, args):
    """The same PMC evidence as pmc_evidence(), collected IN THIS RUN (one GPU): after the timed region,
    rocprofv3 runs child processes of this bench (`--no-cpu --no-train --no-pmc --steps 3 --warmup 1`,
    the same flow, sizes and library), one counter group per pass (`--kernel-trace --pmc` only, no other
    trace domain; each pass in its own process group under a time limit), plus one `--kernel-trace
    --stats` pass of 20 steps whose average duration of the headline kernel is reported beside the HIP-
    event time. Summarised as tools/pmc_summary.py does (FETCH_SIZE doubled, MI355X_MICROARCH.md §HBM).
    Returns (traffic, valu, rocprof) or None when rocprofv3 is absent or any pass fails (the caller then
    falls back to the committed summary, labelled "not this run")."""
    import shutil
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None or any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None  # no profiler, or this bench already runs under one (never nest them)
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-train", "--no-pmc",
            "--D", str(D), "--N", str(N), "--pairs", str(args.pairs), "--dtype", args.dtype]
    if getattr(args, "inverse", False):
        base.append("--inverse")
    work = tempfile.mkdtemp(prefix="enf_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        return _pmc_passes(prof, base, work, N, D, args)
    finally:
        shutil.rmtree(work, ignore_errors=True)


def _pmc_passes(prof, base, work, N, D, args):
    """pmc_live's passes and summary, in the scratch directory `work`. All passes together get PMC_BUDGET_S
    seconds (a good pass takes 5-10 s); each pass is killed at what is left of it."""
    import csv

    deadline = time.monotonic() + PMC_BUDGET_S

    def left():
        return max(1.0, min(90.0, deadline - time.monotonic()))

    per, dur = {}, []
    passes = PMC_PASSES + ((PMC_PASS_F64,) if args.dtype == "f64" else ())
    for i, grp in enumerate(passes):
        if time.monotonic() >= deadline:
            return None
        d = os.path.join(work, f"p{i}")
        rc = _run_group([prof, "--kernel-trace", "--pmc", *grp.split(), "--output-format", "csv", "-d", d, "-o", "run",
                         "--", *base, "--steps", "3", "--warmup", "1"], left(), d + ".log")
        if rc != 0:
            return None
        agg = {}
        with open(os.path.join(d, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if kernel_match(args, r["Kernel_Name"]):
                    key = (r["Dispatch_Id"], r["Counter_Name"])
                    agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
        for (_, c), v in agg.items():
            per.setdefault(c, []).append(v)
        with open(os.path.join(d, "run_kernel_trace.csv")) as f:
            dur += [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(f)
                    if kernel_match(args, r["Kernel_Name"])]
    c = {k: sorted(v)[len(v) // 2] for k, v in per.items()}
    if not dur or not all(k in c for k in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32",
                                           "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY")):
        return None
    dmed = sorted(dur)[len(dur) // 2]
    d = os.path.join(work, "stats")
    if time.monotonic() >= deadline or _run_group([prof, "--kernel-trace", "--stats", "--output-format", "csv", "-d", d,
                                                   "-o", "run", "--", *base, "--steps", "20", "--warmup", "3"],
                                                  left(), d + ".log") != 0:
        return None
    stats = None
    with open(os.path.join(d, "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            if kernel_match(args, r["Name"]):
                stats = {"kernel": r["Name"], "calls": int(r["Calls"]), "average_ms": float(r["AverageNs"]) / 1e6,
                         "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    # the child's timed launches: the last 20 dispatches of the kernel in its trace (the settle launches before
    # them are in the all-calls average above)
    try:
        with open(os.path.join(d, "run_kernel_trace.csv")) as f:
            tr = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                  for r in csv.DictReader(f) if kernel_match(args, r["Kernel_Name"])]
        last = [v for _, v in sorted(tr)[-20:]]
        if stats is not None and last:
            stats = {"kernel": stats["kernel"], "calls": len(last), "average_ms": sum(last) / len(last) / 1e6,
                     "min_ms": min(last) / 1e6, "max_ms": max(last) / 1e6, "of": "the 20 timed launches (kernel trace)",
                     "all_calls": stats["calls"], "all_calls_average_ms": stats["average_ms"]}
    except (OSError, KeyError, ValueError):
        pass
    src = "this run: rocprofv3 --kernel-trace --pmc passes over child runs of this bench (same flow and sizes)"
    hbm = c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024
    traffic = {"bytes_per_launch": hbm, "source": src}
    trans = c["SQ_INSTS_VALU_TRANS_F32"]
    clk = c["GRBM_GUI_ACTIVE"] / 8 / dmed
    cyc = (ISSUE_CYC_FAST * (c["SQ_INSTS_VALU"] - trans) + ISSUE_CYC_TRANS * trans) / 1024.0
    mix = (ISSUE_CYC_MIX_FAST * (c["SQ_INSTS_VALU"] - trans) + ISSUE_CYC_MIX_TRANS * trans) / 1024.0
    valu = {"insts_per_launch": c["SQ_INSTS_VALU"], "trans_insts_per_launch": trans,
            "insts_per_element_pair": c["SQ_INSTS_VALU"] / (N * D * args.pairs / 64.0),
            "issue_cycle_floor_per_simd": cyc, "pmc_effective_clock_ghz": clk, "pmc_kernel_ms": dmed / 1e6,
            "issue_floor_frac": cyc / (clk * dmed), "mix_cost_frac": mix / (clk * dmed),
            "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
            "lds_insts_per_launch": c.get("SQ_INSTS_LDS"), "source": src}
    if args.dtype == "f64" and all(k in c for k in PMC_PASS_F64.split()):
        # the fp64 program: classes per element-pair and the issue floor priced with the fp64 costs (fp64
        # non-transcendental 4.2 cycles, rsq/rcp_f64 13.6, the rest as above)
        epu = N * D * args.pairs / 64.0
        f64 = c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"]
        t64 = c["SQ_INSTS_VALU_TRANS_F64"]
        rest = max(0.0, c["SQ_INSTS_VALU"] - f64 - t64 - trans)
        cyc64 = (ISSUE_CYC_F64 * f64 + ISSUE_CYC_F64_TRANS * t64 + ISSUE_CYC_FAST * rest
                 + ISSUE_CYC_TRANS * trans) / 1024.0
        valu["f64_per_element_pair"] = {
            "fma": c["SQ_INSTS_VALU_FMA_F64"] / epu, "add": c["SQ_INSTS_VALU_ADD_F64"] / epu,
            "mul": c["SQ_INSTS_VALU_MUL_F64"] / epu, "trans": t64 / epu,
            "int32": c["SQ_INSTS_VALU_INT32"] / epu, "int64": c["SQ_INSTS_VALU_INT64"] / epu,
            "other": rest / epu}
        valu["issue_cycle_floor_per_simd"] = cyc64
        valu["issue_floor_frac"] = cyc64 / (clk * dmed)
        valu.pop("mix_cost_frac", None)
    return traffic, valu, stats


def bytes_per_launch_of(N, D, esz):
    """Algorithmic bytes of one flow launch: read X, write Y, write ladj."""
    return N * (2 * D + 1) * esz


def max_over_ranks(values, device, world):
    """Element-wise max over ranks of per-rank values (the timed region's wall time and kernel
    time): the whole job is as slow as its slowest GPU. torch.distributed all-reduce(MAX)
    (RCCL between GPUs; gloo in the CPU tests)."""
    import torch

    t = torch.tensor(values, device=device, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return [float(v) for v in t]


def gather_ranks(value, device, world, rank):
    """Every rank's value (list of world floats), by a sum all-reduce of one-hot slots."""
    import torch

    t = torch.zeros(world, device=device, dtype=torch.float64)
    t[rank] = value
    if world > 1:
        torch.distributed.all_reduce(t)
    return [float(v) for v in t]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--N", type=int, default=10_000_000,
                    help="samples per GPU (--scaling weak, the default) or in all (--scaling strong)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: every rank streams its own N columns (the default line); strong: the N columns are "
                         "split over the ranks in contiguous shards (rank r: [N r/world, N (r+1)/world)), value = N x "
                         "steps / the max-over-ranks time -- the fixed-size reading of the metric's 'N=1e7 at 1/2/4/8 "
                         "GPUs' (VERDICT r05 item 6)")
    ap.add_argument("--pairs", type=int, default=4, help="number of (Householder, Johnson) pairs")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="before the warmup steps, run the flow for this long (wall clock) so that the GPU reaches "
                         "its steady clock: the first ~25 launches of the 0.7 ms headline kernel run 0.86 -> 0.63 ms "
                         "(profiles/r04_bench_order_*.json), longer than the driver's 5 warmup steps; 200 ms leaves a 10x margin "
                         "for nodes whose power management settles more slowly; 0 disables")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-train", action="store_true", help="skip the config-5 training leg (`train` object)")
    ap.add_argument("--train-timeout", type=float, default=240.0,
                    help="several ranks: seconds the training leg may take before the headline line is printed "
                         "without it and the ranks exit")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of each CPU baseline leg")
    ap.add_argument("--pattern", default=None,
                    help="layer letters in application order (S C K J I H, H<k> = k chained reflections), e.g. "
                         "SHK or H4JH4J (overrides --pairs)")
    ap.add_argument("--inverse", action="store_true",
                    help="time inverse(flow) on the forward flow's outputs (what a round trip reads)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the in-run rocprofv3 PMC passes (one GPU; report the committed summary instead)")
    ap.add_argument("--cache", choices=["auto", "warm", "cold", "both"], default="auto",
                    help="cold: every timed step reads and writes its own set of X / Y / ladj buffers, rotating over "
                         "enough sets that more than 1 GiB passes between two uses of a set (the 256 MiB Infinity "
                         "Cache then holds none of it); warm: one set (cache-resident when it is small); both: warm "
                         "then cold, value = cold; auto: both when one set is under 1 GiB, else warm (= cold by size)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="time the K steps as one HIP graph replay (on), or as eager launches with an event between "
                         "launches (off); auto: the graph when one launch moves under 1 GiB (a kernel of tens of "
                         "microseconds, shorter than the host's launch cost), eager otherwise (the headline)")
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="CPU tests only: the launch / barrier / max-over-ranks harness on gloo with a CPU "
                         "stand-in step (measures nothing)")
    args = ap.parse_args()

    # N > 1 started by hand: start the N ranks as child processes before anything touches a GPU
    rc = enf_launch.spawn_ranks_if_needed(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world, rank, local_rank = enf_launch.rank_env()
    enf_launch.check_world(args.gpus, world)
    # stdout carries only the one JSON line: everything else written to file descriptor 1 from here on (RCCL's
    # version banner when a communicator initialises, library prints) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch

    backend = "gloo" if args.selftest_cpu else "nccl"
    if args.selftest_cpu:
        dev = torch.device("cpu")
        if world > 1:
            torch.distributed.init_process_group("gloo")
    else:
        if world > 1:
            torch.cuda.set_device(local_rank)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            torch.cuda.set_device(0)
        dev = torch.device("cuda", torch.cuda.current_device())
    np_dtype = np.float32 if args.dtype == "f32" else np.float64
    t_dtype = torch.float32 if args.dtype == "f32" else torch.float64
    esz = 4 if args.dtype == "f32" else 8
    D = args.D
    strong = args.scaling == "strong"
    # this rank's columns: all N per rank (weak), or its contiguous shard of the N columns (strong)
    N = (args.N * (rank + 1)) // world - (args.N * rank) // world if strong else args.N
    N_total = args.N if strong else args.N * world
    set_bytes = N * (2 * D + 1) * esz  # one launch's X, Y and ladj
    fwd_layers = build_flow(D, args.pairs, np_dtype, pattern=args.pattern)
    layers = invert_layers(fwd_layers) if args.inverse else fwd_layers

    if args.selftest_cpu:
        Xs = np.ones((D, min(N, 4096)), dtype=np_dtype)

        def step():
            np.tanh(Xs).sum()

        def sync():
            pass
        stream = None
    else:
        from enf_pkg import load

        enf = load()
        lib = enf._lib
        L = lib.lib()
        # the shipping library only (diagnostic knobs live in libenf_diag.so, never here)
        assert os.path.basename(lib.loaded_path()) == "libenf.so", lib.loaded_path()
        # synthetic X: N(0,1) columns from torch's counter-based (Philox) CUDA generator; each rank
        # draws its own shard (seed 0x5EED + rank)
        g = torch.Generator(device=dev).manual_seed(0x5EED + rank)
        X = torch.randn((N, D), generator=g, device=dev, dtype=t_dtype)  # row-major N x D == column-major D x N
        Y = torch.empty_like(X)
        ladj = torch.empty(N, device=dev, dtype=t_dtype)
        def layer_array(lays):
            # column-major parameter arrays (a chained Householder V: D x k, Fortran order)
            dps = [[torch.from_numpy(np.ascontiguousarray(np.asarray(p).T)).to(dev) for p in ps] for _, ps in lays]
            a = (lib.Layer * len(lays))()
            for i, ((op, ps), dp) in enumerate(zip(lays, dps)):
                a[i].op = op
                a[i].k = (np.asarray(ps[0]).shape[1] if np.asarray(ps[0]).ndim == 2 else 1) if op == 5 else 0
                for q, t in enumerate(dp):
                    a[i].p[q] = t.data_ptr()
            return a, dps

        arr, dparams = layer_array(layers)
        stream = torch.cuda.current_stream(dev)
        sh = stream.cuda_stream
        dt_code = lib.ENF_F32 if args.dtype == "f32" else lib.ENF_F64
        if args.inverse:
            # the inverse's input is the forward flow's output (untimed): X <- forward(X); each timed step then
            # writes inverse(X) into Y
            farr, fdp = layer_array(fwd_layers)
            lib.check(L.enf_flow_apply(dt_code, D, N, X.data_ptr(), D, Y.data_ptr(), D, ladj.data_ptr(), 0,
                                       farr, len(fwd_layers), sh))
            X, Y = Y, X
            torch.cuda.synchronize()

        # buffer sets for the cold leg: set 0 is (X, Y, ladj); the others are copies of X with their own outputs
        sets = [(X, Y, ladj)]

        def ensure_sets(k):
            while len(sets) < k:
                sets.append((X.clone(), torch.empty_like(Y), torch.empty_like(ladj)))

        cur = {"k": 1, "i": 0}  # sets in rotation, next set

        def step():
            Xs, Ys, Ls = sets[cur["i"] % cur["k"]]
            cur["i"] += 1
            # (torch's current stream: the launch stream, or the capture stream inside a graph capture)
            lib.check(L.enf_flow_apply(dt_code, D, N, Xs.data_ptr(), D, Ys.data_ptr(), D, Ls.data_ptr(), 0,
                                       arr, len(layers), torch.cuda.current_stream(dev).cuda_stream))

        sync = torch.cuda.synchronize

    # settle (round 4): the GPU ramps its clock over the first ~20 ms of sustained load; the flow runs untimed
    # until --settle-ms of wall clock have passed (checked every 8 launches, at most 4000 launches), then the
    # contract's W warmup steps and the K timed steps follow. Reported as "settle" in the line.
    settle = {"ms": 0.0, "launches": 0}
    if args.settle_ms > 0 and not args.selftest_cpu:
        ts = time.perf_counter()
        while settle["launches"] < 4000:
            for _ in range(8):
                step()
            settle["launches"] += 8
            sync()
            if (time.perf_counter() - ts) * 1e3 >= args.settle_ms:
                break
        settle["ms"] = round((time.perf_counter() - ts) * 1e3, 2)
    use_graph = (not args.selftest_cpu) and (args.graph == "on" or (args.graph == "auto" and set_bytes < (1 << 30)))

    def timed(nsets):
        """The contract's W warmup steps and K timed steps (barrier + device sync on both sides) over nsets
        buffer sets in rotation; returns (wall s, mean kernel ms from HIP events, per-launch spread)."""
        if stream is not None:
            cur["k"], cur["i"] = nsets, 0
        for _ in range(args.warmup):
            step()
        sync()
        if world > 1:
            torch.distributed.barrier()
        sync()
        if use_graph:
            # the K timed launches captured once as a HIP graph (on the same buffer-set rotation) and replayed once
            # untimed, then once timed: the event pair measures the device's back-to-back launches without the
            # host's per-call launch cost (~5-8 us per ctypes call here, more than a D = 2 kernel's own time)
            cur["i"] = 0
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg):
                for _ in range(args.steps):
                    step()
            cg.replay()
            sync()
            if world > 1:
                torch.distributed.barrier()
            sync()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            cg.replay()
            e1.record(stream)
            sync()
            if world > 1:
                torch.distributed.barrier()
            sync()
            wall = time.perf_counter() - t0
            del cg
            return wall, e0.elapsed_time(e1) / args.steps, None
        if stream is not None:
            # HIP events on the launch stream (torch.cuda.Event on the stream the kernel is launched on), one
            # between consecutive launches: the per-launch spread besides the mean
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
            ev0, ev1 = evs[0], evs[-1]
        t0 = time.perf_counter()
        if stream is not None:
            ev0.record(stream)
        for i in range(args.steps):
            step()
            if stream is not None:
                evs[i + 1].record(stream)
        sync()
        if world > 1:
            torch.distributed.barrier()
        sync()
        wall = time.perf_counter() - t0
        kern_ms = ev0.elapsed_time(ev1) / args.steps if stream is not None else wall / args.steps * 1e3
        per_launch = None
        if stream is not None:
            seq = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
            pl = sorted(seq)
            per_launch = {"min": pl[0], "median": pl[len(pl) // 2], "max": pl[-1], "launches": len(pl),
                          "in_order": [round(v, 4) for v in seq]}
        return wall, kern_ms, per_launch

    # cache state of the timed launches (a working set under the 256 MiB Infinity Cache read
    # back to back is served on-die, not from HBM)
    mode = args.cache
    big = args.selftest_cpu or set_bytes >= (1 << 30)
    if mode == "auto":
        mode = "warm" if big else "both"
    cache, warm = None, None
    nsets = 1 if args.selftest_cpu else max(1, min(64, -(-(1 << 30) // set_bytes) + 1))
    if mode in ("cold", "both") and nsets > 1:
        ensure_sets(nsets)
    if mode == "both" and nsets > 1:
        w_wall, w_ms, w_pl = timed(1)
        warm = {"ms_per_step": w_wall / args.steps * 1e3, "kernel_ms": w_ms, "kernel_ms_per_launch": w_pl,
                "frac": bytes_per_launch_of(N, D, esz) / (w_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "label": "cache-resident: one buffer set read back to back (not an HBM figure)"}
    if mode in ("cold", "both") and nsets > 1:
        wall, kern_ms, per_launch = timed(nsets)
        rot = nsets * set_bytes
        if rot >= (1 << 30):
            cache = {"mode": "cold", "sets": nsets, "set_MB": set_bytes / 1e6, "rotation_MB": rot / 1e6,
                     "why": "each timed step reads / writes its own buffer set; more than 1 GiB passes between two "
                            "uses of a set, so the 256 MiB Infinity Cache holds none of it"}
        else:
            # (the rotation is capped at 64 sets: a set this small rotates through less than 1 GiB)
            cache = {"mode": "partially warm", "sets": nsets, "set_MB": set_bytes / 1e6, "rotation_MB": rot / 1e6,
                     "why": f"each timed step reads / writes its own buffer set, but only {rot / 1e6:.1f} MB pass "
                            "between two uses of a set" + (" (it fits the 256 MiB Infinity Cache)"
                                                           if rot <= (256 << 20) else "")}
    else:
        wall, kern_ms, per_launch = timed(1)
        cache = {"mode": "warm" if not big else "cold by size", "sets": 1, "set_MB": set_bytes / 1e6,
                 "why": ("one buffer set larger than 1 GiB: the 256 MiB Infinity Cache holds a fraction of it"
                         if big else "one buffer set read back to back: cache-resident, not an HBM figure")}
    t_local, kern_ms_max = max_over_ranks([wall, kern_ms], dev, world)
    per_rank_kernel_ms = gather_ranks(kern_ms, dev, world, rank)
    ms_per_step = t_local / args.steps * 1e3
    total_samples = N_total * args.steps
    value = total_samples / t_local

    bytes_per_launch = bytes_per_launch_of(N, D, esz)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic, valu, rocprof = None, None, None
    if not args.selftest_cpu:
        live = None
        if world == 1 and not args.no_pmc and args.pattern is None and D in (32, 64, 128):
            try:
                live = pmc_live(D, N, args)
            except Exception:  # noqa: BLE001 -- the committed summary below, labelled "not this run"
                live = None
        if live is not None:
            traffic, valu, rocprof = live
        elif not args.inverse:
            traffic, valu = pmc_evidence(D, N, args)
    copy = None if args.selftest_cpu else copy_ceiling(lib, X, Y, stream)
    copy_gbs = copy["GBps"] if copy else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.selftest_cpu and not args.inverse:
        cpu = cpu_baseline(layers, D, np_dtype, args.cpu_seconds)
    headline = (D, N, args.pairs, args.dtype, args.pattern, args.inverse, strong) == (32, 10_000_000, 4, "f32", None,
                                                                                     False, False)
    out = None
    if rank == 0:
        out = {
            "metric": "samples/sec fwd+logdetjac through composed flow, D=32 N=1e7, at 1/2/4/8 GPUs",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": dict(settle, why="untimed launches before the warmup steps until the GPU holds its steady "
                                       "clock (the first ~25 launches ramp 0.86 -> 0.63 ms, "
                                       "profiles/r04_bench_order_*.json)"),
            "ms_per_step": ms_per_step,
            "cache": cache,
            "warm": warm,
            "timing": ("one HIP graph replay of the K launches (events around it; no host launch cost)" if use_graph
                       else "eager launches, HIP events between consecutive launches"),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": ("selftest (CPU stand-in step, measures nothing)" if args.selftest_cpu else
                     "synthetic: X ~ N(0,1) (torch Philox, seed 0x5EED+rank); params seed 42"
                     + ("; the inverse reads forward(X)" if args.inverse else "")),
            "config": {"workload": (f"inverse of {'∘'.join(reversed(layer_letters(fwd_layers)))} = "
                                    if args.inverse else "")
                                   + f"{'∘'.join(reversed(layer_letters(layers)))} composed flow "
                                   + (f"fwd+ladj, D={D}, N={args.N} in all, split over {world} GPU(s)" if strong
                                      else f"fwd+ladj, D={D}, N={N} per GPU"),
                       "D": D, "N_per_gpu": N, "N_total": N_total, "layers": len(layers),
                       "parallelism": f"sample-shard x{world}"},
            "distributed": {"world_size": world, "backend": backend if world > 1 else None,
                            "data_path_collective": None, "per_rank_kernel_ms": per_rank_kernel_ms},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel_ms": kern_ms, "kernel_ms_max_rank": kern_ms_max,
                         "kernel_ms_per_launch": per_launch,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "copy_ceiling_GBps": copy_gbs,
                         "frac_of_copy_ceiling": achieved / copy_gbs if copy_gbs else None,
                         "copy_ceiling": copy,
                         "rocprof_kernel_stats": rocprof},
            "valu": valu,
            "cpu_baseline": cpu,
            "train": None,
        }
    # the config-5 leg after the headline is measured; on several ranks under a watchdog, so that a collective that
    # never completes (libenf's own RCCL communicator) still leaves the headline line, with the train object's error
    if args.selftest_cpu and not args.no_train:  # the config-5 leg's rank plumbing on gloo
        import bench_train

        train = bench_train.train_leg_selftest(world, rank, steps=min(args.steps, 20))
    elif headline and not args.no_train:
        watchdog = None
        if world > 1:
            import threading

            def expire():
                if rank == 0:
                    out["train"] = {"error": f"watchdog: the training leg did not finish in {args.train_timeout:g} s"}
                    print(json.dumps(out), file=json_out, flush=True)
                os._exit(0)  # (no exec: the process ends; the GPU work it left is torn down with it)

            watchdog = threading.Timer(args.train_timeout, expire)
            watchdog.daemon = True
            watchdog.start()
        train = train_leg(dev, world, rank)
        if watchdog is not None:
            watchdog.cancel()
    else:
        train = None
    if rank == 0:
        out["train"] = train
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def train_leg(dev, world, rank):
    """Config 5 (optimize_whitening, D = 32, N = 1e7, B = 1e5, 4x(J∘H), ADAGrad)
    on the same ranks after the headline measurement, reported beside it as the `train` object (its
    own metric, steps/s; not part of `value`). One epoch (100 steps) after 5 warm-up steps, the timed
    steps captured once as a HIP graph and replayed. One rank: the fused step (enf_whitening_step).
    Several ranks: each minibatch split over the ranks, the gradient sums combined by RCCL over xGMI
    called through libenf (EnfComm, enf_allreduce_sum) on the kernels' stream, so gradient, all-reduce
    and update of every step are in the graph (bench_train.py's fastest data-parallel step). Errors are
    reported in the object, never replace the headline."""
    import bench_train

    try:
        res = bench_train.train_leg(dev, world, rank, graph=True, comm_kind="enf", breakdown=True)
    except Exception as e:  # noqa: BLE001 -- the headline line is printed regardless
        return {"error": f"{type(e).__name__}: {e}"}
    if world == 1:
        # one rank's data-parallel step at the 8-GPU share (B/8 = 12 500 columns per step): gradient, single-rank
        # RCCL all-reduce and update, graph-captured, plus its eager per-phase breakdown
        try:
            s8 = bench_train.train_leg(dev, 1, 0, graph=True, comm_kind="enf", emulate_world=8, breakdown=True)
            res["rank_share_of_8"] = {k: s8[k] for k in ("value", "ms_per_step", "step", "launch", "phases", "config")}
            # the same step as three calls (gradient, all-reduce, enf_whitening_apply), with its per-phase breakdown
            u8 = bench_train.train_leg(dev, 1, 0, graph=True, comm_kind="enf", emulate_world=8, breakdown=True,
                                       dp_fused=False)
            res["rank_share_of_8"]["separate_calls"] = {k: u8[k] for k in ("value", "ms_per_step", "step", "phases")}
        except Exception as e:  # noqa: BLE001
            res["rank_share_of_8"] = {"error": f"{type(e).__name__}: {e}"}
        # the reference's own example training loops (examples/nf_example_1d.jl, nf_example_2d.jl: fp64, their
        # flows, minibatch sizes and step counts), each beside the oracle's loop on one host thread
        res["reference_examples"] = {}
        for ex in ("1d", "2d"):
            try:
                res["reference_examples"][ex] = bench_train.example_leg(dev, ex)
            except Exception as e:  # noqa: BLE001
                res["reference_examples"][ex] = {"error": f"{type(e).__name__}: {e}"}
    return res


def copy_ceiling(lib, X, Y, stream, reps=10, settle_ms=100.0):
    """Practical streaming ceiling of this GPU (confirm the HBM peak with a device copy): the
    library's hand-written copy kernel (enf_stream_copy: global_load_dwordx4 / store per lane, 4 or 8 fragments in
    flight per lane, nontemporal or plain) over at least 1 GiB each way, after its own settle run of `settle_ms`,
    timed with HIP events on the launch stream; the best variant is the ceiling (torch's
    copy_ reached 4.6 TB/s where this kernel shape reaches ~6.3 TB/s, MI355X_MICROARCH.md). torch's copy_ of the
    same buffers is reported beside it. Y is overwritten (after the timed steps)."""
    import torch

    nbytes = X.numel() * X.element_size()
    if nbytes < (1 << 30):  # a small flow's buffers would sit in the Infinity Cache: copy a 1 GiB pair instead
        src = torch.empty(1 << 28, dtype=torch.float32, device=X.device).normal_()
        dst = torch.empty_like(src)
        nbytes = src.numel() * 4
    else:
        src, dst = X, Y
    L = lib.lib()
    sh = stream.cuda_stream

    def run(v):
        lib.check(L.enf_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, v, sh))

    ts = time.perf_counter()
    while (time.perf_counter() - ts) * 1e3 < settle_ms:
        for _ in range(4):
            run(0)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    per = {}
    for v in (0, 1, 2, 3):
        for _ in range(2):
            run(v)
        e0.record(stream)
        for _ in range(reps):
            run(v)
        e1.record(stream)
        torch.cuda.synchronize()
        per[v] = 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
    dst.copy_(src)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(reps):
        dst.copy_(src)
    e1.record(stream)
    torch.cuda.synchronize()
    tgbs = 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
    best = max(per, key=per.get)
    names = {0: "4 fragments/lane, nontemporal", 1: "4 fragments/lane, plain", 2: "8 fragments/lane, nontemporal",
             3: "1 fragment/lane, one pass"}
    return {"GBps": per[best], "variant": names[best], "bytes_each_way": nbytes,
            "per_variant_GBps": {names[v]: round(g, 1) for v, g in per.items()}, "torch_copy_GBps": tgbs,
            "kernel": "enf_stream_copy (csrc/enf_copy.hip)"}


def host_info():
    """nproc and the CPU model of this host (lscpu), for the CPU baseline record."""
    import subprocess

    info = {"nproc": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except OSError:
        pass
    q = cgroup_cpu_quota()
    if q is not None:
        info["cgroup_cpu_quota"] = q
    if os.environ.get("OMP_NUM_THREADS"):
        info["OMP_NUM_THREADS"] = os.environ["OMP_NUM_THREADS"]
    return info


def cgroup_cpu_quota():
    """CPUs this process may use per the cgroup CPU bandwidth limit (v2 cpu.max, v1 cfs quota / period),
    rounded up; None when unlimited or unknown. nproc and the affinity mask show the whole machine on a
    shared GPU box, so the CPU baseline sizes its thread count by this."""
    import math

    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, math.ceil(int(quota) / int(period)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            quota = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = int(f.read())
        return max(1, math.ceil(quota / period)) if quota > 0 else None
    except (OSError, ValueError):
        return None


def cpu_baseline(layers, D, np_dtype, seconds):
    """The oracle (CPU restatement of the reference algorithm; Julia is unavailable) timed on a bounded
    sample of the same workload on this host, in two legs of ~`seconds` each: reference-structured,
    1 thread (layer by layer, materialising Y and the D x N ladj temporaries as the Julia broadcasts
    do), and the same arithmetic on all usable host cores (OpenMP column blocks; the affinity mask capped by
    the cgroup CPU quota). The sample size is
    calibrated on a short probe so each leg runs about `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # bench cpu_baseline leg only

    oracle.build()
    info = host_info()
    # every CPU this process may actually use: the affinity mask, capped by the cgroup CPU quota (a shared
    # GPU box shows the whole machine in nproc / the mask; threads beyond the quota only time-slice)
    ncores = info.get("affinity_cpus") or os.cpu_count() or 1
    if info.get("cgroup_cpu_quota"):
        ncores = min(ncores, info["cgroup_cpu_quota"])
    rng = np.random.default_rng(1)
    probe = np.asfortranarray(rng.standard_normal((D, 20_000)).astype(np_dtype))
    t0 = time.perf_counter()
    oracle.flow_apply(layers, probe)
    rate1 = probe.shape[1] / (time.perf_counter() - t0)
    n1 = max(20_000, int(rate1 * seconds))
    X = np.asfortranarray(rng.standard_normal((D, n1)).astype(np_dtype))
    t0 = time.perf_counter()
    oracle.flow_apply(layers, X)
    t1 = time.perf_counter() - t0
    del X
    t0 = time.perf_counter()
    oracle.flow_apply(layers, probe, nthreads=ncores)
    ratem = probe.shape[1] / (time.perf_counter() - t0)
    # a 20k-column probe over hundreds of threads is dominated by thread start-up and underestimates the
    # rate: re-size once from the first full-size run if it was much shorter than the target
    for _ in range(2):
        nm = max(20_000, min(int(ratem * seconds), 50_000_000))
        X = np.asfortranarray(rng.standard_normal((D, nm)).astype(np_dtype))
        t0 = time.perf_counter()
        oracle.flow_apply(layers, X, nthreads=ncores)
        tm = time.perf_counter() - t0
        del X
        ratem = nm / tm
        if tm >= 0.5 * seconds or nm == 50_000_000:
            break
    return {"value": nm / tm, "unit": "samples/s", "cores": ncores, "kind": "port",
            "sample": f"{nm} samples of the same flow (D={D}), CPU restatement of the reference algorithm "
                      f"(Julia unavailable), OpenMP over {ncores} threads, {tm:.1f} s",
            "single_thread": {"value": n1 / t1, "cores": 1, "samples": n1, "seconds": t1,
                              "structure": "reference-structured: layer by layer, D x N ladj temporaries"},
            "host": info}


if __name__ == "__main__":
    main()
