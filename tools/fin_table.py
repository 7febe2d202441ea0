#!/usr/bin/env python3
"""Tabulate a final pass's bench lines (tools/final_r6.sh): python tools/fin_table.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f)[:-5]
    try:
        x = json.load(open(f))
    except (ValueError, OSError):
        continue
    if "roofline" not in x:
        continue
    rp, rg, cb, e2e = x.get("route_pack") or {}, x.get("regroup") or {}, x.get("cpu_baseline") or {}, x.get("e2e") or {}
    print(f"{name:24s} value {x['value']:>10.1f} frac {x['roofline']['frac']:.4f} us {x['roofline']['launch_us']:7.2f} "
          f"layout {x['config'].get('lane_layout', '')[:8]:8s} rp {rp.get('value', '-')!s:>10} pk_ms {rp.get('packing_ms', '-')!s:>6} "
          f"ro_ms {rp.get('route_only_ms', '-')!s:>6} two {(rp.get('two_threads') or {}).get('value', '-')!s:>10} "
          f"rg {rg.get('value', '-')!s:>9} rg_ms {rg.get('ms_per_step', '-')!s:>6} cpu {cb.get('value', '-')!s:>8} "
          f"e2e {e2e.get('value', '-')!s:>8} traffic {x['roofline'].get('traffic')} ceil {x['roofline'].get('read_ceiling', {}).get('achieved')}")
