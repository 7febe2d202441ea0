#!/bin/bash
# Two picks before deferring (SR_KNOB_DEFER_PICKS 2: the general picks kernel) against one (KV_DEFER1),
# route only and route + pack, C3 2 of 4 / C4 7 of 16 / C5 16 of 64 dead, three rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
: > $O/r5s_ab.jsonl
for r in 1 2 3; do
  for cfg in c3 c4 c5; do
    for dp in 1 2; do
      out=$(timeout -k 10 200 python bench.py --config $cfg --dead 0.25 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off --knob defer_picks=$dp 2> $O/r5s_last.err) || { cat $O/r5s_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'picks': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'packing_ms': rp['packing_ms']}))" "$out" $cfg $dp >> $O/r5s_ab.jsonl
    done
  done
done
