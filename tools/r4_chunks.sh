#!/bin/bash
# Round-4 chunk-layout pass: layout tests, the parity suite with every context in the chunk layout
# (SR_LAYOUT=3), then route-only bench lines of C2..C5 in the chunk layout next to AUTO.
# Usage: bash tools/r4_chunks.sh <tag> [configs]
tag=${1:-r4c}; cfgs=${2:-"c2 c5"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_layout_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_layout_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_layout_tests.log
SR_LAYOUT=3 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mtu.py tests/test_gpu_router_core.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/${tag}_parity_chunks.log 2>&1 || { tail -40 gpurun_out/${tag}_parity_chunks.log; exit 1; }
tail -2 gpurun_out/${tag}_parity_chunks.log
for c in $cfgs; do
  for lay in chunks auto; do
    timeout -k 10 300 python bench.py --config $c --layout $lay --no-cpu --no-e2e > gpurun_out/bench_${tag}_${c}_${lay}.json \
      2> gpurun_out/bench_${tag}_${c}_${lay}.err || { tail -20 gpurun_out/bench_${tag}_${c}_${lay}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_${tag}_${c}_${lay}.json')); print('$c $lay', d['value'], d['roofline']['frac'], d['roofline'].get('launch_us'), json.dumps(d.get('route_pack')))"
  done
done
