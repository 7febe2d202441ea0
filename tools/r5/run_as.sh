#!/bin/bash
# Owner pack tiles of 256 records (c1: twice the workgroups; the C5 scatter waits two thirds of its
# cycles with one wave per slot) against 512 (base): regroup parity on c1, then the regroup leg A/B
cd "$(dirname "$0")/../.."
O=gpurun_out
for v in c1; do
  SR_ROUTE_LIB=tools/ab/r5_$v/libsr_route.so timeout -k 10 400 python -u -m pytest tests/test_gpu_regroup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5as_tests_$v.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/r5as_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
: > $O/r5as_ab.jsonl
for r in 1 2; do
  for cfg in c2 c3 c5; do
    for lib in tools/ab/r5_base tools/ab/r5_c1; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $cfg --regroup-steps 32 2> $O/r5as_last.err) || { cat $O/r5as_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); g=d['regroup']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'value': g.get('value'), 'ms': g.get('ms_per_step'), 'err': g.get('error')}))" "$out" $cfg $lib >> $O/r5as_ab.jsonl
    done
  done
done
