#!/bin/bash
# The prefetch code's cost when off: the build before it (tools/ab/r5_hist1d: same all-alive kernels)
# against this one with SR_KNOB_PREFETCH 0 and 64; route only, C2 / C3 / C5, three rounds alternating
cd "$(dirname "$0")/../.."
O=gpurun_out
: > $O/r5j_ab.jsonl
for r in 1 2 3; do
  for cfg in c2 c5 c3; do
    for v in "tools/ab/r5_hist1d -1" "tools/ab/r5_pf 0" "tools/ab/r5_pf 64"; do
      set -- $v
      k=""; [ "$2" != "-1" ] && k="--knob prefetch=$2"
      out=$(SR_ROUTE_LIB=$1/libsr_route.so timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --no-pack --regroup off $k 2> $O/r5j_last.err) || { cat $O/r5j_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'prefetch': int(sys.argv[4]), 'route_us': d['roofline']['launch_us'], 'value': d['value']}))" "$out" $cfg $1 $2 >> $O/r5j_ab.jsonl
    done
  done
done
