#!/bin/bash
# round-6 A/B of the route kernels' prologue: shipped build (base); header in one load + batch by
# selects (v1); header and block-indexed class row in one round trip, scanner granule loaded before
# the epoch (v8)
set -o pipefail
mkdir -p gpurun_out/r6s
bash tools/ab_bench.sh gpurun_out/r6s/ab.jsonl 3 tools/ab/base,tools/ab/v1,tools/ab/v8 "--no-pack --regroup off" "--config c3 --no-pack --regroup off" "--config c4 --no-pack --regroup off" "--config c5 --no-pack --regroup off"
