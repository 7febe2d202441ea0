#!/bin/bash
# round-6 A/B of the route kernels' prologue: shipped build (base); header and block-indexed class row
# in one round trip, then the batch descriptor (v8); the batch sources in the class rows too (v9)
set -o pipefail
mkdir -p gpurun_out/r6t
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py > gpurun_out/r6t/tests.log 2>&1 || { tail -30 gpurun_out/r6t/tests.log; exit 1; }
tail -2 gpurun_out/r6t/tests.log
bash tools/ab_bench.sh gpurun_out/r6t/ab.jsonl 3 tools/ab/base,tools/ab/v8,tools/ab/v9 "--no-pack --regroup off" "--config c3 --no-pack --regroup off" "--config c4 --no-pack --regroup off" "--config c5 --no-pack --regroup off"
