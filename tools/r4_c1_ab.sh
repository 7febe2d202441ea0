#!/bin/bash
# Same-box C1 A/B: this build's statsd-router-mi355x against round 2's data thread
# (tools/ab_r2: the build of 9a15ad4) and the reference executable, over loopback, alternating, two
# rounds per shape. One JSON line per run in gpurun_out/c1_ab_<tag>.jsonl.
# Usage: bash tools/r4_c1_ab.sh <tag> [rounds] [seconds] [extra c1_bench args]
tag=${1:-r4}; rounds=${2:-2}; secs=${3:-3}; shift $(( $# < 3 ? $# : 3 )); extra="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
out="$R/gpurun_out/c1_ab_${tag}.jsonl"
: > "$out"
for r in $(seq 1 "$rounds"); do
  for shape in "1 1" "1 2" "4 3"; do
    set -- $shape
    timeout -k 10 200 python "$R/tools/loopback/c1_bench.py" --threads "$1" --blasters "$2" --seconds $secs \
      --exe "r2=$R/tools/ab_r2/bin/statsd-router-mi355x" $extra \
      >> "$out" 2>> "$R/gpurun_out/c1_ab_${tag}.err" || exit 1
  done
done
python - "$out" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
for r in rows:
    print(f"{r['kind']:10s} threads {r['threads_num']} senders {r['blasters']} offered {r['offered_lines_per_s']/1e6:6.2f} M "
          f"delivered_lines_per_s {r['delivered_lines_per_s']/1e6:6.2f} M fraction {r['delivered_fraction']:.3f} "
          f"tail {r.get('sink_tail_s')}")
PY
