#!/bin/bash
# round-6 A/B of the route kernels' prologue: v8 (shipped: header and block-indexed class row in one
# round trip, then the batch descriptor) against v10 (the kpow and ctl pointers in the first round trip
# too, so the power-table, epoch and scanner-granule loads follow the tile's loads without a wait)
set -o pipefail
mkdir -p gpurun_out/r6v
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py > gpurun_out/r6v/tests.log 2>&1 || { tail -30 gpurun_out/r6v/tests.log; exit 1; }
tail -1 gpurun_out/r6v/tests.log
bash tools/ab_bench.sh gpurun_out/r6v/ab.jsonl 3 tools/ab/v8,tools/ab/v10 "--no-pack --regroup off" "--config c3 --no-pack --regroup off" "--config c4 --no-pack --regroup off" "--config c2 --dead 0.25 --no-pack --regroup off"
