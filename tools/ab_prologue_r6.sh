#!/bin/bash
# round-6 A/B of the chunk kernel's prologue: v8 (shipped) against v11 (the dword before the tile loaded
# unconditionally after the tables, so no wait for the tile's loads precedes the tables' loads)
set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py > gpurun_out/r6w/tests.log 2>&1 || { tail -30 gpurun_out/r6w/tests.log; exit 1; }
tail -1 gpurun_out/r6w/tests.log
bash tools/ab_bench.sh gpurun_out/r6w/ab.jsonl 3 tools/ab/v8,tools/ab/v11 "--config c5 --no-pack --regroup off" "--config c5 --dead 0.25 --no-pack --regroup off" "--config c2 --layout chunks --no-pack --regroup off"
