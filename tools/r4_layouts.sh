#!/bin/bash
# Route-only launch time of every lane layout on the given configs, alternating layouts, <rounds>
# rounds (same box). One JSON line per run in gpurun_out/<tag>_layouts.jsonl, then min per layout.
# Usage: bash tools/r4_layouts.sh <tag> <rounds> "<cfgs>" [extra bench args]
tag=$1; rounds=$2; cfgs=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_layouts.jsonl
: > $out
for r in $(seq 1 "$rounds"); do
  for c in $cfgs; do
    for lay in uniform segments chunks auto; do
      o=$(timeout -k 10 120 python bench.py --config $c --layout $lay --no-cpu --no-e2e --no-pack --regroup off \
          --steps 200 "$@" 2> gpurun_out/${tag}_last.err) || { tail -20 gpurun_out/${tag}_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'layout': sys.argv[2], 'cfg': sys.argv[3], 'launch_us': d['roofline']['launch_us'], 'frac': d['roofline']['frac'], 'captured': d['config'].get('lane_layout')}))" "$o" "$lay" "$c" >> $out
    done
  done
done
python - $out <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); agg[(r["cfg"], r["layout"])].append(r["launch_us"])
for k in sorted(agg): print(k, ["%.1f" % x for x in agg[k]], "min %.1f" % min(agg[k]))
PY
