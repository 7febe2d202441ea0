#!/bin/bash
# KV_DEAD1: N - 1's reciprocal read from LDS on the dead branch (d1l: fewer SGPR spills) against the
# final build: dead-shard parity, then C2 1 of 4 dead route only + route + pack, three rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5aj_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5aj_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5aj_ab.jsonl
for r in 1 2 3; do
  for lib in tools/ab/r5_fin3 tools/ab/r5_d1l; do
    out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config c2 --dead 0.25 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5aj_last.err) || { cat $O/r5aj_last.err; exit 1; }
    python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': 'c2', 'dead': 0.25, 'lib': sys.argv[2], 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $lib >> $O/r5aj_ab.jsonl
  done
done
