#!/bin/bash
# VALU / SALU / LDS instruction counts per route_kernel variant of tools/ablate_route (one
# rocprofv3 --pmc pass per counter group). Usage: tools/pmc_ablate.sh <outdir> [line_len] [quick]
set -e
out=$1; len=${2:-64}; mode=$3
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- tools/ablate_route $len $mode > "$out/p$i.log" 2>&1
done
