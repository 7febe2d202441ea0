#!/bin/bash
# persistent chunk kernel with in-order tile taking: its tests, then C2 / C5 bench lines against the default
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k persist > $O/r5b_persist_tests.log 2>&1
rc=$?; echo "persist tests rc=$rc" >> $O/r5b_persist_tests.log; case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in c2 c5; do
  for k in 0 2; do
    timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --no-pack --knob persist=$k > $O/r5b_bench_${cfg}_persist$k.json 2> $O/r5b_bench_${cfg}_persist$k.err
    rc=$?; echo "bench $cfg persist=$k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
