#!/bin/bash
# Round 5, first GPU pass: the whole GPU suite (new bench-shape, TRACE and fault tests), the default
# bench line, then the persistent chunk kernel (SR_KNOB_PERSIST) tests and bench lines.
# A step that ends in a fault, abort, segfault or time limit ends the script.
cd "$(dirname "$0")/../.."
O=gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: rc=$1"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not persist" > $O/r5a_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5a_gpu_tests.log; ok $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r5a_bench.json 2> $O/r5a_bench.err
rc=$?; echo "bench rc=$rc"; ok $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k persist > $O/r5a_persist_tests.log 2>&1
rc=$?; echo "persist tests rc=$rc" >> $O/r5a_persist_tests.log; ok $rc
for cfg in c2 c5; do
  for k in 0 2; do
    timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --knob persist=$k > $O/r5a_bench_${cfg}_persist$k.json 2> $O/r5a_bench_${cfg}_persist$k.err
    rc=$?; echo "bench $cfg persist=$k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
