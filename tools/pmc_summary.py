#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc_passes.sh for the route kernel.

  python tools/pmc_summary.py <pmc_dir> <config> <out_summary.json> [<out_traffic.json>] [--kernel NAME]

Counters are grouped by the EXACT kernel name rocprofv3 reports (template arguments included), so
route_kernel's and route_chunk_kernel's variants (and AUTO's segment-layout probes) never pool. The
summary describes the variant with the most dispatches (the one the timed launches ran), or the
one whose name contains NAME; the others are listed under "other_kernels" with their own medians.

Per counter: the median over that kernel's dispatches. HBM traffic per launch (one dispatch):
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies wide streaming reads at half their
bytes (MI355X_MICROARCH.md, HBM section), so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact
for 16-B streaming stores (the 8-B record stores are uncalibrated: reported as is).
"""
import csv
import glob
import hashlib
import json
import os
import re
import statistics
import sys

ROUTE_KERNELS = ("route_chunk_kernel", "route_kernel")


def base_name(kn):
    """route_kernel / route_chunk_kernel from a demangled name (None: not a route kernel)."""
    m = re.search(r"\b(route_chunk_kernel|route_kernel)\b", kn)
    return m.group(1) if m else None


def main():
    argv = list(sys.argv[1:])
    want = None
    if "--kernel" in argv:
        i = argv.index("--kernel")
        want = argv[i + 1]
        del argv[i: i + 2]
    d, config, out = argv[0], argv[1], argv[2]
    traffic_out = argv[3] if len(argv) > 3 else None
    vals = {}    # exact kernel name -> counter -> [per-dispatch values]
    metas = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row["Kernel_Name"]
                if base_name(kn) is None:
                    continue
                key = (kn, row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
                metas.setdefault(kn, {"kernel": base_name(kn), "name": kn, "grid_size": int(row["Grid_Size"]),
                                      "workgroup_size": int(row["Workgroup_Size"]),
                                      "lds_bytes": int(row["LDS_Block_Size"]), "vgpr": int(row["VGPR_Count"]),
                                      "sgpr": int(row["SGPR_Count"])})
        for (kn, _, name), v in per.items():
            vals.setdefault(kn, {}).setdefault(name, []).append(v)
    if not vals:
        raise SystemExit(f"no route kernel dispatches under {d}")

    def count(kn):
        return max(len(v) for v in vals[kn].values())

    names = sorted(vals, key=count, reverse=True)
    if want:
        names = [n for n in names if want in n] + [n for n in names if want not in n]
    top = names[0]
    med = {k: statistics.median(v) for k, v in sorted(vals[top].items())}
    res = {"config": config, "kernel": base_name(top), "kernel_name": top, "dispatches": count(top),
           "median_per_dispatch": med, "kernel_meta": metas[top],
           "other_kernels": [{"kernel_name": n, "dispatches": count(n),
                              "median_per_dispatch": {k: statistics.median(v) for k, v in sorted(vals[n].items())}}
                             for n in names[1:]]}
    if "FETCH_SIZE" in med:
        rd = 2.0 * med["FETCH_SIZE"] * 1024
        wr = med.get("WRITE_SIZE", 0.0) * 1024
        res["hbm_read_bytes_per_launch"] = rd
        res["hbm_write_bytes_per_launch"] = wr
        res["hbm_bytes_per_launch"] = rd + wr
    # the build the counters were taken on (bench.py reports them only for the same library)
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "statsd-router_amd", "lib",
                       "libsr_route.so")
    if os.path.exists(lib):
        res["lib_sha256"] = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    if traffic_out and "hbm_bytes_per_launch" in res:
        with open(traffic_out, "w") as fh:
            json.dump({k: res.get(k) for k in ("config", "kernel", "kernel_name", "hbm_bytes_per_launch",
                                               "hbm_read_bytes_per_launch", "hbm_write_bytes_per_launch",
                                               "dispatches", "lib_sha256")}, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "other_kernels"}))


if __name__ == "__main__":
    main()
