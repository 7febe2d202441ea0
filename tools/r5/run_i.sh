#!/bin/bash
# SR_KNOB_PREFETCH: parity with the knob on, then route-only A/B of tiles-ahead 0 / 32 / 64 / 128 / 224
# (C2 uniform, C4 uniform, C5 chunks), two rounds alternating
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_shape.py -m gpu -x -q --timeout 300 --timeout-method thread -k "prefetch" > $O/r5i_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5i_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5i_ab.jsonl
for r in 1 2; do
  for cfg in c2 c5 c4; do
    for pf in 0 32 64 128 224; do
      out=$(timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --no-pack --regroup off --knob prefetch=$pf 2> $O/r5i_last.err) || { cat $O/r5i_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'cfg': sys.argv[2], 'prefetch': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'frac': d['roofline']['frac'], 'layout': d['config'].get('lane_layout')}))" "$out" $cfg $pf >> $O/r5i_ab.jsonl
    done
  done
done
