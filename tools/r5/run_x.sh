#!/bin/bash
# Packing scatter with the keys' positions in registers (no LDS array, no wave syncs per row): parity,
# then route + pack A/B against the build before, C2 / C3 (group scatter), C4 (classic, 17 keys),
# C5 (classic, 65 keys: unchanged path), three rounds; kernel stats on C2 and C4
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mtu.py tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5x_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5x_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5x_ab.jsonl
for r in 1 2 3; do
  for cfg in c2 c3 c4 c5; do
    for lib in tools/ab/r5_base2 tools/ab/r5_sreg tools/ab/r5_sreg2; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5x_last.err) || { cat $O/r5x_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $lib >> $O/r5x_ab.jsonl
    done
  done
done
export TMPDIR=/tmp
R=$(pwd)
for c in c2 c5; do
  (cd /tmp && SR_ROUTE_LIB=$R/tools/ab/r5_sreg2/libsr_route.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5x_prof_$c" -o run \
     -- python "$R/bench.py" --config $c --no-cpu --no-e2e --regroup off --steps 30 --warmup 5 > "$R/$O/r5x_prof_$c.json" 2> "$R/$O/r5x_prof_$c.err") || exit 1
done
