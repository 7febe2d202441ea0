#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes over a route + pack bench command (tools/r4_pmc_pack.sh).

  python tools/pmc_pack_summary.py <pmc_dir> <out.json>

For each packing kernel (mtu_*) and the route kernel: the median over dispatches of every counter,
and the L2 <-> fabric bytes per dispatch: FETCH_SIZE and WRITE_SIZE are KiB. FETCH_SIZE is reported
both raw and doubled (the gfx950 correction of MI355X_MICROARCH.md is calibrated for wide streaming
reads; the packing kernels' 8-byte record reads and u8/u16 arrays are not), WRITE_SIZE as is. The
fabric side includes the MALL, so bytes the scatter wrote and the table kernel reads back may never
reach HBM.
"""
import csv
import glob
import json
import os
import statistics
import sys


def short(kn):
    for k in ("mtu_count_kernel", "mtu_scan_kernel", "mtu_scatter_kernel", "mtu_table_kernel", "mtu_emit_kernel",
              "mtu_chain_kernel", "route_chunk_kernel", "route_kernel", "pack_out_kernel"):
        if k in kn:
            return k
    return None


def main():
    d, out = sys.argv[1], sys.argv[2]
    vals = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if not k:
                    continue
                key = (k, row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        for (k, _, name), v in per.items():
            vals.setdefault(k, {}).setdefault(name, []).append(v)
    res = {}
    for k, cs in sorted(vals.items()):
        med = {n: statistics.median(v) for n, v in sorted(cs.items())}
        r = {"dispatches": max(len(v) for v in cs.values()), "median_per_dispatch": med}
        if "FETCH_SIZE" in med:
            r["fetch_bytes_raw"] = med["FETCH_SIZE"] * 1024
            r["fetch_bytes_x2"] = 2 * med["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in med:
            r["write_bytes"] = med["WRITE_SIZE"] * 1024
        w = med.get("SQ_WAVES") or 0
        if w:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if n in med:
                    r[n.lower().replace("sq_insts_", "") + "_per_wave"] = med[n] / w
        res[k] = r
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, r in res.items():
        print(f"{k:22s} dispatches {r['dispatches']:4d} fetch MB raw {r.get('fetch_bytes_raw', 0) / 1e6:8.1f} "
              f"x2 {r.get('fetch_bytes_x2', 0) / 1e6:8.1f} write MB {r.get('write_bytes', 0) / 1e6:8.1f} "
              f"VALU/wave {r.get('valu_per_wave', 0):7.1f} LDS/wave {r.get('lds_per_wave', 0):6.1f}")


if __name__ == "__main__":
    main()
