#!/bin/bash
# End-of-round refresh on one box (via gpurun, from the repo root): GPU tests, the driver's bench
# command, every config's line (all alive and 25 % dead), rocprofv3 kernel stats of C2 and C5, the C2
# PMC passes (counter traffic for this build), C1 over loopback. Outputs under gpurun_out/fin_*.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
part=${1:-all}
if [ "$part" != "profiles" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin_gpu_tests.log 2>&1 || { tail -30 gpurun_out/fin_gpu_tests.log; exit 1; }
tail -1 gpurun_out/fin_gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin_bench_driver.json 2> gpurun_out/fin_bench_driver.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/fin_bench_c2.json 2> gpurun_out/fin_bench_c2.err || exit 1
for cc in c3 c4 c5 c2dead c4dead c5dead; do
  c=${cc%dead}; extra=""; [ "$c" != "$cc" ] && extra="--dead 0.25"
  timeout -k 10 200 python bench.py --config $c --no-cpu --no-e2e $extra > gpurun_out/fin_bench_$cc.json 2> gpurun_out/fin_bench_$cc.err || exit 1
done
for f in gpurun_out/fin_bench_*.json; do
  python -c "import json,sys; d=json.load(open('$f')); rp=d.get('route_pack') or {}; print('$f', d['value'], d['roofline']['frac'], d['roofline']['launch_us'], 'route_pack', rp.get('value'), rp.get('packing_ms'), (rp.get('two_threads') or {}).get('value'))"
done
fi
[ "$part" = "lines" ] && exit 0
for c in c2 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/fin_prof_$c" -o run \
     -- python "$R/bench.py" --config $c --no-cpu --no-e2e > "$R/gpurun_out/fin_prof_$c.json" 2> "$R/gpurun_out/fin_prof_$c.err") || exit 1
done
tools/pmc_passes.sh gpurun_out/fin_pmc --steps 256 --warmup 16 --config c2 || exit 1
python tools/pmc_summary.py gpurun_out/fin_pmc c2 gpurun_out/fin_pmc_summary_c2.json gpurun_out/fin_pmc_traffic.json > /dev/null || exit 1
for tb in "1 2" "1 3" "4 3"; do
  set -- $tb
  timeout -k 10 120 python tools/loopback/c1_bench.py --only ours --threads $1 --blasters $2 --seconds 3 >> gpurun_out/fin_c1.jsonl 2>> gpurun_out/fin_c1.err || exit 1
done
cat gpurun_out/fin_c1.jsonl
