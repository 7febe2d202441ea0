#!/bin/bash
# One GPU-box pass for this round (from the repo root, via gpurun): GPU tests, the default bench line
# (with the route+pack leg's two-thread measurement), a same-box route+pack A/B of lib dirs, rocprofv3
# kernel stats of the C2 and C5 route+pack legs, C1 over loopback.
# Usage: bash tools/r3_check.sh <tag> [skip-tests] [ab lib dirs...]
tag=${1:-cur}; shift
skip=$1; shift
mkdir -p gpurun_out
if [ "$skip" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
  tail -2 gpurun_out/${tag}_gpu_tests.log
fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_${tag}_c2.json 2> gpurun_out/bench_${tag}_c2.err || { tail -20 gpurun_out/bench_${tag}_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_${tag}_c2.json')); print('c2', d['value'], d['roofline']['frac'], d['roofline']['launch_us'], json.dumps(d.get('route_pack')))"
if [ $# -gt 0 ]; then
  AB_CFGS="c2 c5" bash tools/ab_pack.sh 2 "$@" > gpurun_out/ab_pack_${tag}.txt 2>&1 || { cat gpurun_out/ab_pack_${tag}.txt; exit 1; }
  cat gpurun_out/ab_pack_${tag}.txt
fi
for c in c2 c5; do
  bash tools/prof_stats.sh ${tag}_$c --config $c --no-cpu --no-e2e --steps 50 --regroup off > /dev/null || exit 1
  echo "== $c"; cat gpurun_out/prof_${tag}_$c.txt
done
timeout -k 10 120 python tools/loopback/c1_bench.py --only ours --threads 1 --blasters 2 --seconds 3 > gpurun_out/c1_${tag}.jsonl 2> gpurun_out/c1_${tag}.err || exit 1
cat gpurun_out/c1_${tag}.jsonl
