#!/bin/bash
# Instruction counts per wave of route_kernel under bench.py, one rocprofv3 --pmc pass per config.
# Usage: tools/pmc_valu.sh <outdir> <config>... ; summary: python tools/pmc_summary.py <outdir>/<config> <config> <json>
set -e
out=$1; shift
export TMPDIR=/tmp
for c in "$@"; do
  mkdir -p "$out/$c"
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM \
      --output-format csv -d "$out/$c/p1" -o pmc -- python bench.py --no-cpu --no-e2e --no-pack --regroup off --steps 64 --config $c > "$out/$c/p1.log" 2>&1
done
