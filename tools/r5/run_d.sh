#!/bin/bash
# Route-kernel tile histograms for the packing (sr_route_pack_many): the GPU suite, route-only A/B
# against the build before them, and route + pack with the histograms (hist=1) or the counting pass (hist=0)
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not persist" > $O/r5d_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5d_gpu_tests.log; case $rc in 0|1) ;; *) exit $rc;; esac
rm -f $O/ab.jsonl
AB_CFGS="c2 c3 c4" bash tools/ab_kernels.sh 2 tools/ab/r5_riearly tools/ab/r5_hist > $O/r5d_ab_route.txt 2>&1 || exit $?
mv $O/ab.jsonl $O/r5d_ab_route.jsonl
: > $O/r5d_pack_ab.jsonl
for r in 1 2; do
  for cfg in c2 c3 c4 c5; do
    for h in 0 1; do
      out=$(timeout -k 10 200 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu --no-e2e --knob hist=$h 2> $O/r5d_last.err) || { cat $O/r5d_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'hist': int(sys.argv[3]), 'route_us': d['roofline']['launch_us'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'route_only_ms': rp['route_only_ms'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $h >> $O/r5d_pack_ab.jsonl
    done
  done
done
cat $O/r5d_pack_ab.jsonl
