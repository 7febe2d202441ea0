#!/bin/bash
# Round-4 route-kernel diagnosis on one box: per-tile s_memrealtime stamps (tools/stamps_route) of the
# uniform / segment / chunk layouts, then PMC instruction counts per wave of the bench's C2 launch in
# the chunk and AUTO layouts. Usage: bash tools/r4_diag.sh <tag> [pmc]
tag=${1:-r4d}; want=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for run in "64 4 uni" "64 4 chunks" "0 64 seg" "0 64 chunks" "1024 16 uni" "1024 16 chunks"; do
  set -- $run
  echo "== stamps $run"
  timeout -k 10 120 tools/stamps_route $1 $2 $3 > gpurun_out/${tag}_stamps_$1_$3.txt 2>&1 || { cat gpurun_out/${tag}_stamps_$1_$3.txt; exit 1; }
  grep -v residency gpurun_out/${tag}_stamps_$1_$3.txt
done
if [ "$want" = "pmc" ]; then
  bash tools/r4_pmc.sh ${tag}chunks c2 --layout chunks || exit 1
  bash tools/r4_pmc.sh ${tag}auto c2 --layout auto || exit 1
fi
