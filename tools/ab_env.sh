#!/bin/bash
# Same-box A/B of SR_STAGGER settings (the route kernel's staggered first round) on the bench's
# route-only line: bash tools/ab_env.sh <rounds> "<setting>" ... (setting "" = off); AB_CFGS as in
# ab_kernels.sh. Prints µs per 32-batch launch.
rounds=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for st in "$@"; do
    for c in ${AB_CFGS:-c2 c5}; do
      out=$(SR_STAGGER="$st" timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --no-verify --no-pack --regroup off --steps 400 2>gpurun_out/ab_last.err) || { cat gpurun_out/ab_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print('stagger=%-10s' % sys.argv[2], sys.argv[3], d['roofline']['launch_us'], d['roofline']['frac'])" "$out" "$st" "$c"
    done
  done
done
