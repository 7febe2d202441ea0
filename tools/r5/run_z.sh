#!/bin/bash
# Kernel stats of the regroup leg (C5 and C2, own chunk in place), one GPU
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
R=$(pwd)
for c in c5 c2; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5z_prof_$c" -o run \
     -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $c --regroup-steps 32 > "$R/$O/r5z_prof_$c.json" 2> "$R/$O/r5z_prof_$c.err") || exit 1
done
