#!/bin/bash
# Dead-shard route A/B of several builds of libsr_route.so (same box, alternating): route-only launch
# time and route + pack with 25 % of the shards dead.
# Usage: bash tools/r4_dead3.sh <tag> <rounds> "<cfgs>" <lib dir>...
tag=$1; rounds=$2; cfgs=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_dead.jsonl
: > $out
for r in $(seq 1 "$rounds"); do
  for c in $cfgs; do
    for lib in cur "$@"; do
      libpath=$R/statsd-router_amd/lib/libsr_route.so
      [ "$lib" != "cur" ] && libpath=$R/$lib/libsr_route.so
      o=$(SR_ROUTE_LIB=$libpath timeout -k 10 200 python bench.py --config $c --dead 0.25 --no-cpu --no-e2e \
          --regroup off --steps 100 2> gpurun_out/${tag}_last.err) || { tail -20 gpurun_out/${tag}_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'lib': sys.argv[2], 'cfg': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'route_pack': rp['value'], 'packing_ms': rp['packing_ms']}))" "$o" "$lib" "$c" >> $out
    done
  done
done
python - $out <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); agg[(r["cfg"], r["lib"])].append((r["route_us"], r["route_pack"]))
for k in sorted(agg): print(k, "route_us", [x[0] for x in agg[k]], "route+pack", [x[1] for x in agg[k]])
PY
