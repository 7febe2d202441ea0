#!/bin/bash
# Uniform kernel: the record base read at the window start (ABL_EARLY_BASE) instead of part-way
# through the first hash; route only, C2 / C3 / C4, three rounds alternating with this build
cd "$(dirname "$0")/../.."
O=gpurun_out
: > $O/r5w_ab.jsonl
for r in 1 2 3; do
  for cfg in c2 c3 c4; do
    for lib in tools/ab/r5_base2 tools/ab/r5_early; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --no-pack --regroup off 2> $O/r5w_last.err) || { cat $O/r5w_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'value': d['value']}))" "$out" $cfg $lib >> $O/r5w_ab.jsonl
    done
  done
done
