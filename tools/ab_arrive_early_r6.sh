#!/bin/bash
# round-6 A/B: tiles arrive right after reading the epoch (earr) instead of at their end (base, shipped)
set -o pipefail
mkdir -p gpurun_out/r6ah
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py > gpurun_out/r6ah/tests.log 2>&1 || { tail -30 gpurun_out/r6ah/tests.log; exit 1; }
tail -1 gpurun_out/r6ah/tests.log
bash tools/ab_bench.sh gpurun_out/r6ah/ab.jsonl 3 tools/ab/base,tools/ab/earr "--no-pack --regroup off --no-verify" "--config c3 --no-pack --regroup off --no-verify" "--config c5 --no-pack --regroup off --no-verify"
