#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc_passes.sh for route_kernel.

  python tools/pmc_summary.py <pmc_dir> <config> <out_summary.json> [<out_traffic.json>]

Per counter: the median over route_kernel dispatches. HBM traffic per launch (one dispatch):
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies wide streaming reads at half their
bytes (MI355X_MICROARCH.md, HBM section), so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact
for 16-B streaming stores (the 8-B record stores are uncalibrated: reported as is).
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, config, out = sys.argv[1], sys.argv[2], sys.argv[3]
    traffic_out = sys.argv[4] if len(sys.argv) > 4 else None
    vals = {}
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row["Kernel_Name"]
                if "route_kernel" not in kn and "route_chunk_kernel" not in kn:
                    continue
                meta.setdefault("kernel", "route_chunk_kernel" if "route_chunk_kernel" in kn else "route_kernel")
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
                meta.setdefault("grid_size", int(row["Grid_Size"]))
                meta.setdefault("workgroup_size", int(row["Workgroup_Size"]))
                meta.setdefault("lds_bytes", int(row["LDS_Block_Size"]))
                meta.setdefault("vgpr", int(row["VGPR_Count"]))
                meta.setdefault("sgpr", int(row["SGPR_Count"]))
        for (_, name), v in per.items():
            vals.setdefault(name, []).append(v)
    med = {k: statistics.median(v) for k, v in sorted(vals.items())}
    res = {"config": config, "kernel": meta.get("kernel", "route_kernel"), "dispatches": max((len(v) for v in vals.values()), default=0),
           "median_per_dispatch": med, "kernel_meta": meta}
    if "FETCH_SIZE" in med:
        rd = 2.0 * med["FETCH_SIZE"] * 1024
        wr = med.get("WRITE_SIZE", 0.0) * 1024
        res["hbm_read_bytes_per_launch"] = rd
        res["hbm_write_bytes_per_launch"] = wr
        res["hbm_bytes_per_launch"] = rd + wr
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    # the build the counters were taken on (bench.py reports them only for the same library)
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "statsd-router_amd", "lib",
                       "libsr_route.so")
    if os.path.exists(lib):
        res["lib_sha256"] = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    if traffic_out and "hbm_bytes_per_launch" in res:
        with open(traffic_out, "w") as fh:
            json.dump({k: res.get(k) for k in ("config", "kernel", "hbm_bytes_per_launch", "hbm_read_bytes_per_launch",
                                               "hbm_write_bytes_per_launch", "dispatches", "lib_sha256")}, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
