#!/bin/bash
# round-6 A/B of the packing kernels' batch lookups: v11 (lane-per-batch vector loads of the kernel
# argument) against v12 (scalar loads, all issued before the first compare)
set -o pipefail
mkdir -p gpurun_out/r6x
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mtu.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py tests/test_gpu_regroup.py > gpurun_out/r6x/tests.log 2>&1 || { tail -30 gpurun_out/r6x/tests.log; exit 1; }
tail -1 gpurun_out/r6x/tests.log
bash tools/ab_bench.sh gpurun_out/r6x/ab.jsonl 3 tools/ab/v11,tools/ab/v12 "--regroup off --no-verify" "--config c5 --regroup off --no-verify" "--config c3 --regroup off --no-verify"
