#!/bin/bash
# Round-4 baseline pass on one box: the default bench line (C2) and C5, route-only, then the C1 A/B.
# Usage: bash tools/r4_base.sh <tag>
tag=${1:-r4base}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R" || exit 1
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err \
    || { tail -20 gpurun_out/bench_${tag}_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${tag}_$c.json')); print('$c', d['value'], d['roofline']['frac'], d['roofline'].get('launch_us'), json.dumps(d.get('route_pack')))"
done
bash tools/r4_c1_ab.sh "$tag" 2
