#!/bin/bash
# Owner pack: pk7 (batch by ballot, coalesced scan) and pk8 (+ flat 16-byte piece copy) against the committed build: regroup parity, then the
# regroup leg A/B (C2 64-byte lines, C3 256, C5 mixed), two rounds, and a profile of pk8
cd "$(dirname "$0")/../.."
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_regroup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5ag_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/r5ag_tests.log; [ $rc -eq 0 ] || exit $rc
: > $O/r5ag_ab.jsonl
for r in 1 2; do
  for cfg in c2 c3 c5; do
    for lib in tools/ab/r5_one tools/ab/r5_pk7 tools/ab/r5_pk8; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $cfg --regroup-steps 32 2> $O/r5ag_last.err) || { cat $O/r5ag_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); g=d['regroup']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'value': g.get('value'), 'ms': g.get('ms_per_step'), 'err': g.get('error')}))" "$out" $cfg $lib >> $O/r5ag_ab.jsonl
    done
  done
done
export TMPDIR=/tmp
R=$(pwd)
for c in c2 c5; do
  (cd /tmp && SR_ROUTE_LIB=$R/tools/ab/r5_pk8/libsr_route.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5ag_prof_$c" -o run \
     -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $c --regroup-steps 32 > "$R/$O/r5ag_prof_$c.json" 2> "$R/$O/r5ag_prof_$c.err") || exit 1
done
