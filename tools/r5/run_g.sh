#!/bin/bash
# Regroup: the own chunk written straight into the receive buffer. Regroup parity suites, then the
# regroup leg A/B (in place vs the round-4 pack + copy) on C5 and C2, 32 steps, two rounds
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_regroup.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/r5g_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5g_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5g_regroup_ab.jsonl
for r in 1 2; do
  for cfg in c5 c2; do
    for mode in inplace copy; do
      extra=""; [ $mode = copy ] && extra="--regroup-copy-own"
      out=$(timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $cfg --regroup-steps 32 $extra 2> $O/r5g_last.err) || { cat $O/r5g_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); g=d['regroup']; print(json.dumps({'cfg': sys.argv[2], 'mode': sys.argv[3], 'value': g.get('value'), 'ms': g.get('ms_per_step'), 'err': g.get('error')}))" "$out" $cfg $mode >> $O/r5g_regroup_ab.jsonl
    done
  done
done
# kernel stats of the route + pack leg (C2, C5) on this build
export TMPDIR=/tmp
R=$(pwd)
for c in c2 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5g_prof_$c" -o run \
     -- python "$R/bench.py" --config $c --no-cpu --no-e2e --regroup off --steps 50 --warmup 10 > "$R/$O/r5g_prof_$c.json" 2> "$R/$O/r5g_prof_$c.err") || exit 1
done
