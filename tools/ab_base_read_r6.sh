#!/bin/bash
# round-6 A/B: the record base read at the window start as well as part-way through the hash, the
# first valid of the two used (v13), against the part-way read alone (v11, shipped)
set -o pipefail
mkdir -p gpurun_out/r6y
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py > gpurun_out/r6y/tests.log 2>&1 || { tail -30 gpurun_out/r6y/tests.log; exit 1; }
tail -1 gpurun_out/r6y/tests.log
bash tools/ab_bench.sh gpurun_out/r6y/ab.jsonl 3 tools/ab/v11,tools/ab/v13 "--no-pack --regroup off" "--config c3 --no-pack --regroup off" "--config c4 --no-pack --regroup off" "--config c2 --dead 0.25 --no-pack --regroup off"
