#!/bin/bash
# Same-box A/B of library builds: bash tools/ab_kernels.sh <rounds> <lib dir A> <lib dir B> ... (each holding
# libsr_route.so; "<dir>@<layout>" also passes --layout <layout> to bench.py); bench lines for c2..c5
# alternate between the builds. Output: gpurun_out/ab.jsonl. AB_CFGS overrides the configs ("c2 c4dead ...": a
# trailing "dead" runs the config with 25 % of the shards dead).
rounds=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for d in "$@"; do
    for cc in ${AB_CFGS:-c2 c3 c4 c5}; do
      lib=${d%@*}; extra=""
      [ "$lib" != "$d" ] && extra="--layout ${d#*@}"
      c=${cc%dead}; [ "$c" != "$cc" ] && extra="$extra --dead 0.25"
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --no-verify --no-pack --regroup off --steps 400 $extra 2>gpurun_out/ab_last.err) || { cat gpurun_out/ab_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'lib': sys.argv[2], 'cfg': sys.argv[3], 'frac': d['roofline']['frac'], 'launch_us': d['roofline']['launch_us'], 'layout': d['config'].get('lane_layout')}))" "$out" "$d" "$cc" >> gpurun_out/ab.jsonl
    done
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/ab.jsonl")]
agg = collections.defaultdict(list)
for r in rows: agg[(r["lib"], r["cfg"])].append(r["launch_us"])
for k in sorted(agg): print(k, ["%.1f" % v for v in agg[k]], "min %.1f" % min(agg[k]))
PY
