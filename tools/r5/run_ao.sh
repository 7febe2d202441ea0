#!/bin/bash
# Owner scatter: byte-aligned 16-byte loads (ua; ua2 with copy batch 2) against the realigned dword loads
# (the final build, and cb2): regroup parity on ua and ua2, then the regroup leg A/B (C2, C3, C5), two rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
for v in ua ua2; do
  SR_ROUTE_LIB=tools/ab/r5_$v/libsr_route.so timeout -k 10 400 python -u -m pytest tests/test_gpu_regroup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5ao_tests_$v.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/r5ao_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
: > $O/r5ao_ab.jsonl
for r in 1 2; do
  for cfg in c2 c3 c5; do
    for lib in tools/ab/r5_fin3 tools/ab/r5_cb2 tools/ab/r5_ua tools/ab/r5_ua2; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $cfg --regroup-steps 32 2> $O/r5ao_last.err) || { cat $O/r5ao_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); g=d['regroup']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'value': g.get('value'), 'ms': g.get('ms_per_step'), 'err': g.get('error')}))" "$out" $cfg $lib >> $O/r5ao_ab.jsonl
    done
  done
done
