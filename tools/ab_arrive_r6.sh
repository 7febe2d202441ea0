#!/bin/bash
# round-6 A/B of the launch's arrival counters: 8 counters (v11, shipped), 64 counters on separate
# lines (arr64), and the timing bound with no tile arrivals at all (arr: -DSR_ABL_LEAN_ARRIVE)
set -o pipefail
mkdir -p gpurun_out/r6aa
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py > gpurun_out/r6aa/tests.log 2>&1 || { tail -30 gpurun_out/r6aa/tests.log; exit 1; }
tail -1 gpurun_out/r6aa/tests.log
bash tools/ab_bench.sh gpurun_out/r6aa/ab.jsonl 3 tools/ab/v11,tools/ab/arr64,tools/ab/arr "--no-pack --regroup off --no-verify" "--config c3 --no-pack --regroup off --no-verify" "--config c5 --no-pack --regroup off --no-verify"
