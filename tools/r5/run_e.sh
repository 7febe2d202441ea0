#!/bin/bash
# Tile histograms, second version (16-entry scan rounds, 8-tile groups, row-bounded group scatter):
# the packing's GPU tests, then route + pack with hist=1 / hist=0 alternating
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py tests/test_gpu_mtu.py tests/test_gpu_router_core.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not persist" > $O/r5e_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5e_tests.log; case $rc in 0) ;; *) exit $rc;; esac
: > $O/r5e_pack_ab.jsonl
for r in 1 2 3; do
  for cfg in c2 c3 c4; do
    for h in 0 1; do
      out=$(timeout -k 10 200 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu --no-e2e --knob hist=$h 2> $O/r5e_last.err) || { cat $O/r5e_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'hist': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'route_only_ms': rp['route_only_ms'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $h >> $O/r5e_pack_ab.jsonl
    done
  done
done
