#!/bin/bash
# End-of-session refresh on one box: the default bench line + rocprofv3 stats + PMC of C2
# (tools/gpu_profile.sh), every config's bench line, and the C5 PMC summary.
set -e
bash tools/gpu_profile.sh c2 skip-tests
bash tools/bench_configs.sh r2f > gpurun_out/bench_configs_r2f.txt 2>&1
tools/pmc_passes.sh gpurun_out/pmc_c5 --steps 256 --warmup 16 --config c5
python tools/pmc_summary.py gpurun_out/pmc_c5 c5 gpurun_out/pmc_summary_c5.json > /dev/null
