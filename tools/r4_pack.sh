#!/bin/bash
# Round-4 packing pass: the MTU parity tests (default chunk rule, then forced 2048- and 4096-line
# chunks), then route + pack bench lines alternating $VARIANTS (name:ENV=V ..., default this build
# against round 3's table kernel), then rocprofv3 kernel-trace summaries of the route + pack lines.
# Usage: bash tools/r4_pack.sh <tag> [rounds] [configs]
tag=${1:-r4p}; rounds=${2:-2}; cfgs=${3:-"c2 c5"}
VARIANTS=${VARIANTS:-"new: r3:SR_MTU_TABLE=r3"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_mtu.py tests/test_gpu_router_core.py > gpurun_out/${tag}_tests.log 2>&1 \
  || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for envs in SR_MTU_CH=2048 SR_MTU_CH=4608 SR_MTU_WALK=0; do
  env $envs timeout -k 10 300 $T tests/test_gpu_mtu.py tests/test_gpu_router_core.py > gpurun_out/${tag}_tests_$envs.log 2>&1 \
    || { tail -40 gpurun_out/${tag}_tests_$envs.log; exit 1; }
  echo "$envs: $(tail -1 gpurun_out/${tag}_tests_$envs.log)"
done
out=gpurun_out/${tag}_pack.jsonl
: > $out
for r in $(seq 1 "$rounds"); do
  for c in $cfgs; do
    for v in $VARIANTS; do
      name=${v%%:*}; envs=${v#*:}
      o=$(env $envs timeout -k 10 200 python bench.py --config $c --no-cpu --no-e2e --regroup off --steps 50 \
          2> gpurun_out/${tag}_last.err) || { tail -20 gpurun_out/${tag}_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'v': sys.argv[2], 'cfg': sys.argv[3], 'value': rp['value'], 'packing_ms': rp['packing_ms'], 'route_only_ms': rp['route_only_ms'], 'packets': rp['packets_per_launch']}))" "$o" "$name" "$c" >> $out
    done
  done
done
python - $out <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); agg[(r["cfg"], r["v"])].append((r["packing_ms"], r["value"], r["packets"]))
for k in sorted(agg): print(k, "packing_ms", [x[0] for x in agg[k]], "route+pack M/s", [x[1] for x in agg[k]], "packets", agg[k][0][2])
PY
export TMPDIR=/tmp
for c in $cfgs; do
  d=gpurun_out/${tag}_prof_$c
  rm -rf $d
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o prof -- python bench.py --config $c --no-cpu --no-e2e \
      --regroup off --steps 20 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  f=$(find $d -name '*kernel_stats.csv' | head -1)
  python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print("%-60s calls %6s avg_us %8.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
