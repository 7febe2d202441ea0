#!/bin/bash
# PMC passes of the regroup leg's C5 command on the shipped build (for the owner scatter's counters)
cd "$(dirname "$0")/../.."
bash tools/pmc_passes.sh gpurun_out/r5ar_pmc_rg_c5 --steps 3 --warmup 1 --no-pack --regroup on --regroup-config c5 --regroup-steps 16
