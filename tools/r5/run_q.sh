#!/bin/bash
# Tile histograms in the KV_DEAD1 variants (one dead shard): parity, then route + pack A/B against the
# KV_DEAD1 build without them, C2 1 of 4 dead, three rounds alternating
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py tests/test_gpu_mtu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5q_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5q_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5q_ab.jsonl
for r in 1 2 3; do
  for lib in tools/ab/r5_k1 tools/ab/r5_k1h; do
    out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config c2 --dead 0.25 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5q_last.err) || { cat $O/r5q_last.err; exit 1; }
    python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': 'c2', 'lib': sys.argv[2], 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $lib >> $O/r5q_ab.jsonl
  done
done
