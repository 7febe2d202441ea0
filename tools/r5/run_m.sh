#!/bin/bash
# Group scatter: route tiles per wave 4 / 8 (shipped) / 16; route + pack C2 / C3, three rounds
# alternating; kernel stats on C2
cd "$(dirname "$0")/../.."
O=gpurun_out
: > $O/r5m_ab.jsonl
for r in 1 2 3; do
  for cfg in c2 c3; do
    for lib in tools/ab/r5_g4 tools/ab/r5_g8 tools/ab/r5_g16; do
      out=$(SR_ROUTE_LIB=$lib/libsr_route.so timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu --no-e2e --regroup off 2> $O/r5m_last.err) || { cat $O/r5m_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print(json.dumps({'cfg': sys.argv[2], 'lib': sys.argv[3], 'route_us': d['roofline']['launch_us'], 'rp_value': rp['value'], 'rp_ms': rp['ms_per_launch'], 'packing_ms': rp['packing_ms'], 'verify': bool(rp.get('verify'))}))" "$out" $cfg $lib >> $O/r5m_ab.jsonl
    done
  done
done
export TMPDIR=/tmp
R=$(pwd)
for lib in r5_g4 r5_g16; do
  (cd /tmp && SR_ROUTE_LIB=$R/tools/ab/$lib/libsr_route.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5m_prof_$lib" -o run \
     -- python "$R/bench.py" --config c2 --no-cpu --no-e2e --regroup off --steps 30 --warmup 5 > "$R/$O/r5m_prof_$lib.json" 2> "$R/$O/r5m_prof_$lib.err") || exit 1
done
