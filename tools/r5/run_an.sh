#!/bin/bash
# Owner scatter copy batch 2 / 8 (cb2, cb8) against 4 (the final build): regroup parity, then the
# regroup leg A/B (C2 64-byte lines, C3 256, C5 mixed), two rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_regroup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5an_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5an_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5an_ab.jsonl
for r in 1 2; do
  for cfg in c2 c3 c5; do
    for lib in tools/ab/r5_fin3 tools/ab/r5_cb2 tools/ab/r5_cb8; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $cfg --regroup-steps 32 2> $O/r5an_last.err) || { cat $O/r5an_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); g=d['regroup']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'value': g.get('value'), 'ms': g.get('ms_per_step'), 'err': g.get('error')}))" "$out" $cfg $lib >> $O/r5an_ab.jsonl
    done
  done
done
