#!/bin/bash
# KV_DEAD1 (exactly one dead shard: two picks in closed form): the dead-shard parity suites, then
# route + pack A/B against the KV_DEFER1 build, C2 / C3 1 of 4 dead, C5 1 of 64 dead
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mtu.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py tests/test_gpu_layout.py tests/test_gpu_router_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5p_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5p_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5p_ab.jsonl
for r in 1 2 3; do
  for v in "c2 0.25" "c3 0.25" "c5 0.01"; do
    set -- $v
    for lib in tools/ab/r5_d1 tools/ab/r5_k1; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $1 --dead $2 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5p_last.err) || { cat $O/r5p_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'dead': sys.argv[3], 'lib': sys.argv[4], 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $1 $2 $lib >> $O/r5p_ab.jsonl
    done
  done
done
