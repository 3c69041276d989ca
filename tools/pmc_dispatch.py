"""Per-dispatch PMC summary: duration, effective clock (GRBM_GUI_ACTIVE / XCDs / duration) and counters."""
import collections, csv, glob, sys
root, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "flow_"
agg = collections.defaultdict(dict)
meta = {}
for p in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if pat not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        agg[d][r["Counter_Name"]] = agg[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["VGPR_Count"], r["Kernel_Name"][:60])
for d in sorted(agg):
    c, (dur, vg, name) = agg[d], meta[d]
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / dur if dur else 0
    valu = c.get("SQ_ACTIVE_INST_VALU", 0)
    busy = c.get("SQ_BUSY_CYCLES", 0)
    print(f"disp {d:3d} {dur/1000:8.1f} us clk {clk:5.2f} GHz vgpr {vg} VALU insts {c.get('SQ_INSTS_VALU',0):.3e} "
          f"trans {c.get('SQ_INSTS_VALU_TRANS_F32',0):.3e} active_valu {valu:.3e} thread_cyc_valu {c.get('SQ_THREAD_CYCLES_VALU',0):.3e} "
          f"busy {busy:.3e} wave_cyc {c.get('SQ_WAVE_CYCLES',0):.3e} wait_inst {c.get('SQ_WAIT_INST_ANY',0):.3e}")
