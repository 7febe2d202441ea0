#!/usr/bin/env python3
"""Tabulate tools/ab_bench.sh output: per (args, lib), the route launch (us), route + pack and regroup rates."""
import collections
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = (r["ab_args"], r["ab_lib"])
    rp, rg = r.get("route_pack") or {}, r.get("regroup") or {}
    agg[k]["launch_us"].append(r["roofline"]["launch_us"])
    agg[k]["value"].append(r["value"])
    if rp:
        agg[k]["rp_value"].append(rp.get("value"))
        agg[k]["packing_ms"].append(rp.get("packing_ms"))
        if rp.get("two_threads"):
            agg[k]["two_threads"].append(rp["two_threads"]["value"])
    if rg.get("value"):
        agg[k]["regroup"].append(rg["value"])
        agg[k]["regroup_ms"].append(rg.get("ms_per_step"))
for k in sorted(agg):
    print(k[0], "|", k[1])
    for m, v in agg[k].items():
        print("   %-12s %s" % (m, " ".join(str(x) for x in v)))
