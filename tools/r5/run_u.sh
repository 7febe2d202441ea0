#!/bin/bash
# Per-tile phase stamps of the all-alive chunk kernel (tools/stamps_route, s_memrealtime) on 64-byte,
# 1024-byte and mixed lines, and of the uniform kernel on 64-byte lines
cd "$(dirname "$0")/../.."
O=gpurun_out
: > $O/r5u_stamps.txt
for run in "64 4 chunks" "1024 16 chunks" "0 64 chunks" "64 4 uni" "1024 16 uni"; do
  set -- $run
  echo "== $run" >> $O/r5u_stamps.txt
  timeout -k 10 120 tools/stamps_route $1 $2 $3 > $O/r5u_one.txt 2>&1 || { cat $O/r5u_one.txt; exit 1; }
  grep -v residency $O/r5u_one.txt >> $O/r5u_stamps.txt
done
cat $O/r5u_stamps.txt
