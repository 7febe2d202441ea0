#!/bin/bash
# round-6 A/B: the scanner with one count poll in flight (p1, -DSR_SCAN_POLLS1) against two (v11, shipped)
set -o pipefail
mkdir -p gpurun_out/r6ae
SR_ROUTE_LIB=tools/ab/p1/libsr_route.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py > gpurun_out/r6ae/tests.log 2>&1 || { tail -30 gpurun_out/r6ae/tests.log; exit 1; }
tail -1 gpurun_out/r6ae/tests.log
bash tools/ab_bench.sh gpurun_out/r6ae/ab.jsonl 3 tools/ab/v11,tools/ab/p1 "--no-pack --regroup off --no-verify" "--config c3 --no-pack --regroup off --no-verify" "--config c5 --no-pack --regroup off --no-verify"
