#!/bin/bash
# Size exchange by a publish kernel and a host spin (no copies, no stream synchronisation; one rank: no
# collective): regroup parity, then the regroup leg, one call and split (C2, C3, C5), two rounds, trace
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_regroup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5ae_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5ae_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5ae_ab.jsonl
for r in 1 2; do
  for cfg in c2 c3 c5; do
    for mode in one split; do
      extra=""; [ $mode = split ] && extra="--regroup-split-calls"
      out=$(timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $cfg --regroup-steps 32 $extra 2> $O/r5ae_last.err) || { cat $O/r5ae_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); g=d['regroup']; print(json.dumps({'cfg': sys.argv[2], 'mode': sys.argv[3], 'value': g.get('value'), 'ms': g.get('ms_per_step'), 'err': g.get('error')}))" "$out" $cfg $mode >> $O/r5ae_ab.jsonl
    done
  done
done
export TMPDIR=/tmp
R=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5ae_prof_c2" -o run \
   -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config c2 --regroup-steps 32 > "$R/$O/r5ae_prof_c2.json" 2> "$R/$O/r5ae_prof_c2.err") || exit 1
