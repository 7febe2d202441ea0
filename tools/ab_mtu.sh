#!/bin/bash
# Phase timing of the MTU packing kernels: bash tools/ab_mtu.sh <rounds> <config> <lib dir> ... (each holding
# a libsr_route.so built with -DSR_MTU_SKIP=<mask>, see mtu_kernel.hpp); the bench's route+pack leg per
# build, alternating. Output: gpurun_out/ab_mtu.jsonl
rounds=$1; cfg=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for d in "$@"; do
    out=$(SR_ROUTE_LIB=$d/libsr_route.so timeout -k 10 120 python bench.py --config $cfg --no-cpu --no-e2e --no-verify --regroup off --steps 5 --warmup 2 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'lib': sys.argv[2], 'cfg': sys.argv[3], 'packing_ms': d['route_pack']['packing_ms']}))" "$out" "$d" "$cfg" >> gpurun_out/ab_mtu.jsonl
  done
done
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/ab_mtu.jsonl")]
agg = collections.defaultdict(list)
for r in rows: agg[(r["cfg"], r["lib"])].append(r["packing_ms"])
for k in sorted(agg): print(k, ["%.4f" % v for v in agg[k]], "min %.4f" % min(agg[k]))
PY
