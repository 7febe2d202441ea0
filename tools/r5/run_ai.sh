#!/bin/bash
# Kernel traces of route + pack with dead shards (C2 1 of 4, C3 2 of 4) and C2 all alive, this build
cd "$(dirname "$0")/../.."
O=gpurun_out
export TMPDIR=/tmp
R=$(pwd)
for cd in "c2 0.25" "c3 0.25" "c2 0"; do
  set -- $cd
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5ai_prof_$1_$2" -o run \
     -- python "$R/bench.py" --config $1 --dead $2 --steps 20 --warmup 5 --no-cpu --no-e2e --regroup off > "$R/$O/r5ai_prof_$1_$2.json" 2> "$R/$O/r5ai_prof_$1_$2.err") || exit 1
done
