#!/bin/bash
# Bench lines for every configuration on one box (outputs under gpurun_out/bench_<tag>.json).
# Usage (from the repo root, via gpurun): bash tools/bench_configs.sh [tag] [extra bench args...]
tag=${1:-cur}; shift
mkdir -p gpurun_out
for c in c2 c3 c4 c5; do
  timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e "$@" > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err || exit 1
done
timeout -k 10 120 python bench.py --config c2 --dead 0.25 --no-cpu --no-e2e "$@" > gpurun_out/bench_${tag}_c2dead.json 2> gpurun_out/bench_${tag}_c2dead.err || exit 1
for f in gpurun_out/bench_${tag}_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['frac'], d['roofline']['launch_us'])"; done
