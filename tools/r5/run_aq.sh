#!/bin/bash
# The shipped build: three default bench runs in a row (run-to-run spread on one box) and the PMC passes of
# the C5 command (the chunk kernel's HBM traffic and instruction mix)
cd "$(dirname "$0")/../.."
O=gpurun_out
for k in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/r5aq_default_$k.json 2> $O/r5aq_default_$k.err || { tail -20 $O/r5aq_default_$k.err; exit 1; }
done
bash tools/r4_pmc.sh r5aq c5 || exit 1
