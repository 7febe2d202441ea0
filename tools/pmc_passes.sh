#!/bin/bash
# PMC passes for route_kernel under bench.py: one rocprofv3 run per counter group (--pmc is never
# combined with tracing domains). Usage: tools/pmc_passes.sh <outdir> [bench args...]
# Summarise with: python tools/pmc_summary.py <outdir> <config> <summary.json> [traffic.json]
set -e
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- python bench.py --no-cpu --no-e2e "$@" > "$out/p$i.log" 2>&1
done
