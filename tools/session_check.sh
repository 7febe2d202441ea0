#!/bin/bash
# One GPU-box check of the current tree: GPU tests, every config's bench line (route + route_pack
# legs, all alive and 25 % dead), and C1 over loopback (ours, 1 data thread, 2 senders).
# Usage (from the repo root, via gpurun): bash tools/session_check.sh <tag> [skip-tests]
tag=${1:-cur}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
  tail -2 gpurun_out/${tag}_gpu_tests.log
fi
for c in c2 c3 c4 c5; do
  timeout -k 10 150 python bench.py --config $c --no-cpu --no-e2e > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err || exit 1
done
for c in c2 c4 c5; do
  timeout -k 10 150 python bench.py --config $c --dead 0.25 --no-cpu --no-e2e > gpurun_out/bench_${tag}_${c}dead.json 2> gpurun_out/bench_${tag}_${c}dead.err || exit 1
done
for f in gpurun_out/bench_${tag}_*.json; do
  python -c "import json,sys; d=json.load(open('$f')); rp=d.get('route_pack',{}); print('$f', d['value'], d['roofline']['frac'], d['roofline']['launch_us'], 'route_pack', rp.get('value'), rp.get('packing_ms'), rp.get('probed_dead_shards'))"
done
timeout -k 10 120 python tools/loopback/c1_bench.py --only ours --threads 1 --blasters 2 --seconds 3 > gpurun_out/c1_${tag}.jsonl 2> gpurun_out/c1_${tag}.err || exit 1
cat gpurun_out/c1_${tag}.jsonl
