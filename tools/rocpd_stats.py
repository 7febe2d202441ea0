#!/usr/bin/env python3
"""Per-kernel dispatch statistics from a rocprofv3 rocpd database (the ROCm 7 default output, run_results.db),
in the columns of rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs. Optional output csv.

  python tools/rocpd_stats.py <run_results.db> [out.csv]
"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in con.execute("PRAGMA table_info(kernels)")]
    name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    if name is None or "start" not in cols or "end" not in cols:
        raise SystemExit(f"unexpected kernels view columns: {cols}")
    rows = con.execute(f"SELECT {name}, COUNT(*), SUM(end - start), AVG(end - start), MIN(end - start), "
                       f"MAX(end - start) FROM kernels GROUP BY {name} ORDER BY SUM(end - start) DESC").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    for n, c, s, a, mn, mx in rows:
        out.append([n, c, s, round(a, 1), round(100.0 * s / total, 3), mn, mx])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in out[:25]:
        print(",".join(str(x) for x in [r[0][:70]] + r[1:]))


if __name__ == "__main__":
    main()
