#!/bin/bash
# Same-box A/B of the route+pack leg: bash tools/ab_pack.sh <rounds> <lib dir A> <lib dir B> ...; AB_CFGS as in
# ab_kernels.sh ("c5dead": 25 % of the shards dead). Prints route_pack ms per launch, route-only ms, packing ms.
rounds=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for d in "$@"; do
    for cc in ${AB_CFGS:-c2 c5 c2dead c5dead}; do
      c=${cc%dead}; extra=""; [ "$c" != "$cc" ] && extra="--dead 0.25"
      out=$(SR_ROUTE_LIB=$d/libsr_route.so timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --no-verify --regroup off --steps 50 $extra 2>gpurun_out/ab_last.err) || { cat gpurun_out/ab_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1])['route_pack']; print(sys.argv[2], sys.argv[3], 'route_pack_ms', d['ms_per_launch'], 'route_only_ms', d['route_only_ms'], 'packing_ms', d['packing_ms'], 'M/s', d['value'])" "$out" "$d" "$cc"
    done
  done
done
