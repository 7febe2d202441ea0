#!/bin/bash
# One dead shard after the packing's ballot lookups: route + pack with the KV_DEAD1 | KV_HIST1 route kernel
# (hist=1, the shipped path) against KV_DEAD1 + the counting pass (hist=0), C2 1 of 4 dead,
# three rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
: > $O/r5al_ab.jsonl
for r in 1 2 3; do
  for cfg in c2; do
    for h in 1 0; do
      out=$(timeout -k 10 200 python bench.py --config $cfg --dead 0.25 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off --knob hist=$h 2> $O/r5al_last.err) || { cat $O/r5al_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'hist': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $h >> $O/r5al_ab.jsonl
    done
  done
done
