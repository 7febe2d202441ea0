#!/bin/bash
# Deferred-probe picks A/B (SR_DEFER_PICKS=1 / 2) with 25 % of the shards dead, same box, alternating.
# Usage: bash tools/r4_picks_ab.sh <tag> <rounds> "<cfgs>"
tag=$1; rounds=$2; cfgs=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_picks.jsonl
: > $out
for r in $(seq 1 "$rounds"); do
  for c in $cfgs; do
    for k in 1 2; do
      o=$(SR_DEFER_PICKS=$k timeout -k 10 200 python bench.py --config $c --dead 0.25 --no-cpu --no-e2e --regroup off \
          --steps 100 2> gpurun_out/${tag}_last.err) || { tail -20 gpurun_out/${tag}_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'picks': sys.argv[2], 'cfg': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'route_pack': rp['value'], 'packing_ms': rp['packing_ms']}))" "$o" "$k" "$c" >> $out
    done
  done
done
python - $out <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); agg[(r["cfg"], r["picks"])].append((r["route_us"], r["route_pack"]))
for k in sorted(agg): print(k, "route_us", [x[0] for x in agg[k]], "route+pack", [x[1] for x in agg[k]])
PY
