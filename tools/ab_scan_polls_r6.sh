#!/bin/bash
# round-6 A/B: the scanner with four count polls in flight (p4, -DSR_SCAN_POLLS4) against two (v11, shipped)
set -o pipefail
mkdir -p gpurun_out/r6ac
SR_ROUTE_LIB=tools/ab/p4/libsr_route.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py > gpurun_out/r6ac/tests.log 2>&1 || { tail -30 gpurun_out/r6ac/tests.log; exit 1; }
tail -1 gpurun_out/r6ac/tests.log
bash tools/ab_bench.sh gpurun_out/r6ac/ab.jsonl 3 tools/ab/v11,tools/ab/p4 "--no-pack --regroup off --no-verify" "--config c3 --no-pack --regroup off --no-verify" "--config c5 --no-pack --regroup off --no-verify"
