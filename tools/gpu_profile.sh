#!/bin/bash
# One GPU-box session: GPU parity tests, the default bench line, the rocprofv3 kernel-trace/stats
# of the same bench command, and the PMC passes + summary. Outputs under gpurun_out/.
# Usage (from the repo root, via gpurun): bash tools/gpu_profile.sh [config] [skip-tests]
cfg=${1:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd "$R" || exit 1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || exit 1
fi
timeout -k 10 300 python bench.py --config $cfg > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench \
    -- python "$R/bench.py" --config $cfg > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err" && \
cd "$R" && tools/pmc_passes.sh gpurun_out/pmc --steps 256 --warmup 16 --config $cfg && \
python tools/pmc_summary.py gpurun_out/pmc $cfg gpurun_out/pmc_summary.json gpurun_out/pmc_traffic.json > /dev/null
