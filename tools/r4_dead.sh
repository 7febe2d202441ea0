#!/bin/bash
# Dead-shard A/B: route + pack bench lines with 25 % of the shards dead and all
# alive, this build against another build of libsr_route.so (same box, alternating).
# Usage: bash tools/r4_dead.sh <tag> <rounds> "<cfgs>" <other lib dir>
tag=$1; rounds=$2; cfgs=$3; other=$4
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_dead.jsonl
: > $out
for r in $(seq 1 "$rounds"); do
  for c in $cfgs; do
    for lib in cur $other; do
      libpath=$R/statsd-router_amd/lib/libsr_route.so
      [ "$lib" != "cur" ] && libpath=$R/$lib/libsr_route.so
      for dead in 0.25 0; do
        o=$(SR_ROUTE_LIB=$libpath timeout -k 10 200 python bench.py --config $c --dead $dead --no-cpu --no-e2e \
            --regroup off --steps 100 2> gpurun_out/${tag}_last.err) || { tail -20 gpurun_out/${tag}_last.err; exit 1; }
        python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'lib': sys.argv[2], 'cfg': sys.argv[3], 'dead': sys.argv[4], 'route_us': d['roofline']['launch_us'], 'route_pack': rp['value'], 'route_only_ms': rp['route_only_ms'], 'packing_ms': rp['packing_ms'], 'probed_dead': rp['probed_dead_shards']}))" "$o" "$lib" "$c" "$dead" >> $out
      done
    done
  done
done
cat $out
