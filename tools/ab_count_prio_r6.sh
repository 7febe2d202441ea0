#!/bin/bash
# round-6 A/B: the tile's load-to-count phase at raised wave priority (pr1 / pr2: s_setprio 1 / 2 until the
# count is published, -DSR_COUNT_PRIO) against the shipped build (base)
set -o pipefail
mkdir -p gpurun_out/r6ag
bash tools/ab_bench.sh gpurun_out/r6ag/ab.jsonl 3 tools/ab/base,tools/ab/pr1,tools/ab/pr2 "--no-pack --regroup off --no-verify" "--config c3 --no-pack --regroup off --no-verify" "--config c4 --no-pack --regroup off --no-verify"
