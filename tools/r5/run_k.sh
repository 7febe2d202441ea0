#!/bin/bash
# Chunk kernel ablations on this round's build: without the Suf computations, without U (timing and
# C5 instruction counts only; wrong records by design)
cd "$(dirname "$0")/../.."
PMC_CFG=c5 bash tools/r5/abl.sh r5k 2 "c5 c4" cur@cur@chunks nosuf@tools/ab/r5_nosuf@chunks nou@tools/ab/r5_nou@chunks
# prefetch distance on the chunk kernel: C5 all alive and 16 of 64 dead
: > gpurun_out/r5k_pf.jsonl
for r in 1 2; do
  for d in 0 0.25; do
    for pf in 48 64 96 128; do
      out=$(timeout -k 10 200 python bench.py --config c5 --dead $d --steps 100 --warmup 10 --no-cpu --no-e2e --no-pack --regroup off --knob prefetch=$pf 2> gpurun_out/r5k_last.err) || { cat gpurun_out/r5k_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'dead': sys.argv[2], 'prefetch': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'value': d['value']}))" "$out" $d $pf >> gpurun_out/r5k_pf.jsonl
    done
  done
done
