#!/usr/bin/env python3
"""Per-variant medians (per dispatch and per wave) from tools/pmc_ablate.sh output."""
import csv
import glob
import json
import os
import re
import statistics
import sys


def main():
    d = sys.argv[1]
    per = {}
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        acc = {}
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if "route_kernel" not in name and "read_kernel" not in name:
                continue
            m = re.search(r"route_kernel<(\d+), (\d+)u>", name)
            key = f"b{m.group(1)}_abl{m.group(2)}" if m else "read_kernel"
            k2 = (key, row["Dispatch_Id"], row["Counter_Name"])
            acc[k2] = acc.get(k2, 0.0) + float(row["Counter_Value"])
        for (key, _, cn), v in acc.items():
            per.setdefault(key, {}).setdefault(cn, []).append(v)
    res = {}
    for key, cs in sorted(per.items()):
        med = {cn: statistics.median(v) for cn, v in cs.items()}
        w = med.get("SQ_WAVES", 0) or 1
        res[key] = {cn: round(v / w, 1) for cn, v in med.items() if cn != "SQ_WAVES"}
        res[key]["waves"] = w
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
