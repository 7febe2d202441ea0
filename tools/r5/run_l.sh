#!/bin/bash
# mtu_scan with the key starts in LDS (r5_scan), and group scatter: 32 records per lane and round (one round for a C2 group of 8 route tiles, 4 waves
# per SIMD) against 16 (two rounds); route + pack, C2 / C3, three rounds alternating; kernel stats
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 env SR_ROUTE_LIB=tools/ab/r5_scan_grp32/libsr_route.so python -u -m pytest tests/test_gpu_bench_shape.py -m gpu -x -q --timeout 300 --timeout-method thread -k "route_pack_many" > $O/r5l_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5l_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5l_ab.jsonl
for r in 1 2 3; do
  for cfg in c2 c3; do
    for lib in tools/ab/r5_grp16 tools/ab/r5_scan tools/ab/r5_scan_grp32; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5l_last.err) || { cat $O/r5l_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $lib >> $O/r5l_ab.jsonl
    done
  done
done
export TMPDIR=/tmp
R=$(pwd)
for lib in r5_grp16 r5_scan r5_scan_grp32; do
  (cd /tmp && SR_ROUTE_LIB=$R/tools/ab/$lib/libsr_route.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5l_prof_$lib" -o run \
     -- python "$R/bench.py" --config c2 --no-cpu --no-e2e --regroup off --steps 30 --warmup 5 > "$R/$O/r5l_prof_$lib.json" 2> "$R/$O/r5l_prof_$lib.err") || exit 1
done
