#!/bin/bash
# round-6 A/B: status / base granules one per 128-B line (gs16, -DSR_GRAN_STRIDE=16) against packed
# 8-B granules (v11 shipped; gs1 = the same source built with stride 1)
set -o pipefail
mkdir -p gpurun_out/r6ad
SR_ROUTE_LIB=tools/ab/gs16/libsr_route.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py > gpurun_out/r6ad/tests.log 2>&1 || { tail -30 gpurun_out/r6ad/tests.log; exit 1; }
tail -1 gpurun_out/r6ad/tests.log
bash tools/ab_bench.sh gpurun_out/r6ad/ab.jsonl 3 tools/ab/v11,tools/ab/gs1,tools/ab/gs16 "--no-pack --regroup off --no-verify" "--config c3 --no-pack --regroup off --no-verify" "--config c5 --no-pack --regroup off --no-verify"
