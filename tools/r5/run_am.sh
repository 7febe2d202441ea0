#!/bin/bash
# The scatter writing the sorted lengths (2 B per line) for mtu_table (slen) against the final build:
# packing parity, then route + pack A/B (C2, C3, C5, C2 1 of 4 dead), two rounds, and kernel profiles
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py tests/test_gpu_router_core.py tests/test_gpu_mtu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r5am_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5am_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5am_ab.jsonl
for r in 1 2; do
  for cd in "c2 0" "c3 0" "c5 0" "c2 0.25"; do
    set -- $cd
    for lib in tools/ab/r5_fin3 tools/ab/r5_slen; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $1 --dead $2 --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5am_last.err) || { cat $O/r5am_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[3], 'dead': sys.argv[4], 'lib': sys.argv[2], 'route_us': d['roofline']['launch_us'], 'value': d['value'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $lib $1 $2 >> $O/r5am_ab.jsonl
    done
  done
done
export TMPDIR=/tmp
R=$(pwd)
for c in c2 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5am_prof_$c" -o run \
     -- python "$R/bench.py" --config $c --steps 20 --warmup 5 --no-cpu --no-e2e --regroup off > "$R/$O/r5am_prof_$c.json" 2> "$R/$O/r5am_prof_$c.err") || exit 1
done
