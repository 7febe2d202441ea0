#!/bin/bash
# Same-box A/B of environment settings of the library (SR_STAGGER, SR_DEFER_PICKS, ...):
# bash tools/ab_env.sh <rounds> "<VAR=value ...>" ... ("" = defaults); AB_CFGS as in ab_kernels.sh
# ("c5dead": 25 % of the shards dead). Prints µs per 32-batch route launch (timed region, the
# deferred-probe kernel included) and the route+pack leg's ms per launch.
rounds=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for st in "$@"; do
    for cc in ${AB_CFGS:-c2 c5}; do
      c=${cc%dead}; extra=""; [ "$c" != "$cc" ] && extra="--dead 0.25"
      out=$(env $st timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --no-verify --regroup off --steps 300 $extra 2>gpurun_out/ab_last.err) || { cat gpurun_out/ab_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d.get('route_pack') or {}; print('%-22s' % (sys.argv[2] or 'default'), sys.argv[3], 'route_us', d['roofline']['launch_us'], 'frac', d['roofline']['frac'], 'route_pack_ms', rp.get('ms_per_launch'), 'packing_ms', rp.get('packing_ms'))" "$out" "$st" "$cc"
    done
  done
done
