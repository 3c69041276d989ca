"""Median effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md) and VALU count of the
flow_hj_kernel dispatches in a rocprofv3 --kernel-trace --pmc CSV directory (design probe). argv: dirs."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not cc:
        print(d, "no counter csv")
        continue
    per, durs = {}, {}
    for r in csv.DictReader(open(cc[0])):
        if "flow_hj_kernel" not in r["Kernel_Name"]:
            continue
        k = r["Dispatch_Id"]
        per.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        durs[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows = []
    for k, c in per.items():
        rows.append((c.get("GRBM_GUI_ACTIVE", 0) / 8 / durs[k], durs[k] / 1e6, c))
    rows.sort(key=lambda x: x[1])
    clk, ms, c = rows[len(rows) // 2]
    print(f"{d}: {len(rows)} dispatches, median kernel {ms:.4f} ms, clock {clk:.3f} GHz, counters {c}")
