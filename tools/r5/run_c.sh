#!/bin/bash
# chunk kernel: R/RI loads at tile entry (A/B against the committed build, chunk layout), then the
# regroup leg (C5 and C2, 32 batches per step) on this build
cd "$(dirname "$0")/../.."
rm -f gpurun_out/ab.jsonl
AB_CFGS="c5 c2 c4 c5dead" bash tools/ab_kernels.sh 2 tools/ab/r5_base@chunks tools/ab/r5_riearly@chunks > gpurun_out/r5c_ab.txt 2>&1 || exit $?
mv gpurun_out/ab.jsonl gpurun_out/r5c_ab_riearly.jsonl
for cfg in c5 c2; do
  timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --no-verify --regroup on --regroup-config $cfg --regroup-steps 8 > gpurun_out/r5c_regroup_$cfg.json 2> gpurun_out/r5c_regroup_$cfg.err || exit $?
done
