"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv) for one kernel."""
import collections
import csv
import glob
import json
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "flow_frag"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc"
# optional metadata k=v (D=32 N=10000000 dtype=f32 pairs=4 kernel=... git=...): bench.py matches D/N/dtype/pairs
meta = {}
for kv in sys.argv[3:]:
    k, _, v = kv.partition("=")
    meta[k] = int(v) if v.isdigit() else v
per = collections.defaultdict(list)
dur = []
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(p)):
        if pat not in r["Kernel_Name"]:
            continue
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in agg.items():
        per[c].append(v)
for p in sorted(glob.glob(f"{root}/p*/run_kernel_trace.csv")):
    for r in csv.DictReader(open(p)):
        if pat in r["Kernel_Name"]:
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {c: sorted(v)[len(v) // 2] for c, v in per.items()}
out["median_duration_ns_profiled"] = sorted(dur)[len(dur) // 2] if dur else None
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    # gfx950: FETCH_SIZE reports half the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM)
    out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
if "GRBM_GUI_ACTIVE" in out and dur:
    out["effective_clock_ghz"] = out["GRBM_GUI_ACTIVE"] / 8 / out["median_duration_ns_profiled"]
if "SQ_WAVE_CYCLES" in out:
    w = out["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in out:
            out[k + "_frac"] = out[k] / w
if meta:
    counters = {k: v for k, v in out.items() if k.isupper()}
    derived = {k: v for k, v in out.items() if not k.isupper()}
    algo = meta.get("N", 0) * (2 * meta.get("D", 0) + 1) * (4 if meta.get("dtype") == "f32" else 8)
    out = dict(meta, source="rocprofv3 --kernel-trace --pmc, one counter group per pass (tools/pmc.sh); FETCH_SIZE "
                            "doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half of wide coalesced reads)",
               algorithmic_bytes_per_launch=algo, counters=counters, **derived)
print(json.dumps(out, indent=1))
