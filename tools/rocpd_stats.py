"""Kernel statistics (the columns of rocprofv3's --stats CSV) from a rocprofv3 SQLite database (run_results.db,
the default --output-format of this ROCm's rocprofv3): per kernel name the call count, total / average / min /
max duration in ns and the share of the total.

    python tools/rocpd_stats.py gpurun_out/prof_inv/run_results.db profiles/r04_inverse_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(db, out):
    con = sqlite3.connect(db)
    rows = con.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                       "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, a, b in rows:
        agg.setdefault(name, []).append(b - a)
    tot = sum(sum(v) for v in agg.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 6), round(100 * sum(v) / tot, 2), min(v), max(v),
                        round(statistics.pstdev(v), 6)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
