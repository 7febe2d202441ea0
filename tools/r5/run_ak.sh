#!/bin/bash
# Fused deferral re-measured after the ballot batch lookups (mtu_count<FD> no longer waits on a batch loop):
# parity, then route + pack A/B with SR_KNOB_FUSE_DEFER 1 / 0 on this build (C3 2 of 4, C4 7 of 16, C5 16 of 64 dead),
# three rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py tests/test_gpu_mtu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5ak_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5ak_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5ak_ab.jsonl
for r in 1 2 3; do
  for cfg in c3 c4 c5; do
    for fd in 0 1; do
      out=$(timeout -k 10 200 python bench.py --config $cfg --dead 0.25 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off --knob fuse_defer=$fd 2> $O/r5ak_last.err) || { cat $O/r5ak_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'fuse': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $fd >> $O/r5ak_ab.jsonl
    done
  done
done
