#!/bin/bash
# PMC passes of the route + pack bench line (one rocprofv3 --pmc run per counter group, no tracing),
# summarised per kernel by tools/pmc_pack_summary.py into gpurun_out/<tag>_pmc_pack_<cfg>.json.
# Usage: bash tools/r4_pmc_pack.sh <tag> [config]
tag=${1:-r4}; cfg=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
out=gpurun_out/${tag}_pmc_pack_$cfg
rm -rf "$out"
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- \
    python bench.py --config "$cfg" --no-cpu --no-e2e --regroup off --steps 10 --warmup 2 > "$out/p$i.log" 2>&1 \
    || { tail -20 "$out/p$i.log"; exit 1; }
done
python tools/pmc_pack_summary.py "$out" gpurun_out/${tag}_pmc_pack_$cfg.json
