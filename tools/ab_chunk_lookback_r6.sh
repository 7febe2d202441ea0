#!/bin/bash
# round-6 A/B: the chunk kernel's first record-base look-back reads requested right after its count is
# published (v14) instead of when the records are due (v11, shipped)
set -o pipefail
mkdir -p gpurun_out/r6ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py > gpurun_out/r6ab/tests.log 2>&1 || { tail -30 gpurun_out/r6ab/tests.log; exit 1; }
tail -1 gpurun_out/r6ab/tests.log
bash tools/ab_bench.sh gpurun_out/r6ab/ab.jsonl 3 tools/ab/v11,tools/ab/v14 "--config c5 --no-pack --regroup off --no-verify" "--config c5 --dead 0.25 --no-pack --regroup off --no-verify" "--config c2 --layout chunks --no-pack --regroup off --no-verify"
