#!/bin/bash
# Chunk kernel: the predecessor's tail granules read with the record-base reads. Layout / parity
# suites, route-only A/B against the build before (C5, C5 dead, C4 and C2 in the chunk layout),
# three rounds, then the stamps of mixed lines
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_bench_shape.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5v_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5v_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5v_ab.jsonl
for r in 1 2 3; do
  for v in "c5 0 auto" "c5 0.25 auto" "c4 0 chunks" "c2 0 chunks"; do
    set -- $v
    for lib in tools/ab/r5_base2 tools/ab/r5_lbe; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $1 --dead $2 --layout $3 --steps 100 --warmup 10 --no-cpu --no-e2e --no-pack --regroup off 2> $O/r5v_last.err) || { cat $O/r5v_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'cfg': sys.argv[2], 'dead': sys.argv[3], 'layout': sys.argv[4], 'lib': sys.argv[5], 'route_us': d['roofline']['launch_us'], 'value': d['value']}))" "$out" $1 $2 $3 $lib >> $O/r5v_ab.jsonl
    done
  done
done
timeout -k 10 120 tools/stamps_route 0 64 chunks > $O/r5v_stamps.txt 2>&1 || exit 1
