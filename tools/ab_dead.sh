#!/bin/bash
# A/B of C2 and C2 with 25 % dead: bash /tmp/ab_dead.sh rounds libdirs...
rounds=$1; shift
for r in $(seq 1 $rounds); do for d in "$@"; do for a in "" "--dead 0.25" "--config c5 --dead 0.25"; do
  out=$(SR_ROUTE_LIB=$d/libsr_route.so timeout -k 10 120 python bench.py $a --no-cpu --no-e2e --no-verify --no-pack --regroup off --steps 300 2>/dev/null) || exit 1
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], sys.argv[3], d['roofline']['launch_us'])" "$out" "$d" "$a"
done; done; done
