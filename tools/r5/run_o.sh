#!/bin/bash
# KV_DEFER1 (dead-shard variants with the one-pick probe and the alive word as a kernel argument):
# the dead-shard parity suites, then route + pack A/B against the build before, C4 / C5 with 25 % dead
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mtu.py tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py tests/test_gpu_layout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5o_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5o_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5o_ab.jsonl
for r in 1 2 3; do
  for cfg in c4 c5; do
    for lib in tools/ab/r5_g8 tools/ab/r5_d1; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $cfg --dead 0.25 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5o_last.err) || { cat $O/r5o_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $lib >> $O/r5o_ab.jsonl
    done
  done
done
