#!/bin/bash
# round-6 A/B: tile-side look-back for the record base (lb1) against the scanner base alone (v8)
set -o pipefail
mkdir -p gpurun_out/r6u
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py > gpurun_out/r6u/tests.log 2>&1 || { tail -30 gpurun_out/r6u/tests.log; exit 1; }
tail -1 gpurun_out/r6u/tests.log
bash tools/ab_bench.sh gpurun_out/r6u/ab.jsonl 3 tools/ab/v8,tools/ab/lb1 "--no-pack --regroup off" "--config c3 --no-pack --regroup off" "--config c4 --no-pack --regroup off" "--config c2 --dead 0.25 --no-pack --regroup off"
