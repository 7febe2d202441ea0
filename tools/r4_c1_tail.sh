#!/bin/bash
# C1 span diagnosis: this build and round 2's data thread (tools/ab_r2), one data thread, one and two
# senders, with the sink's head / tail against the senders' clocks.
# Usage: bash tools/r4_c1_tail.sh <tag> [rounds] [seconds]
tag=${1:-r4t}; rounds=${2:-2}; secs=${3:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
out="$R/gpurun_out/c1_tail_${tag}.jsonl"
: > "$out"
for r in $(seq 1 "$rounds"); do
  for shape in "1 1" "1 2" "4 3"; do
    set -- $shape
    timeout -k 10 200 python "$R/tools/loopback/c1_bench.py" --threads "$1" --blasters "$2" --seconds $secs --only ours \
      --exe "r2=$R/tools/ab_r2/bin/statsd-router-mi355x" >> "$out" 2>> "$R/gpurun_out/c1_tail_${tag}.err" || exit 1
  done
done
python - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f"{r['kind']:6s} threads {r['threads_num']} senders {r['blasters']} offered {r['offered_lines_per_s']/1e6:6.2f} "
          f"delivered_lines_per_s {r['delivered_lines_per_s']/1e6:6.2f} per_blast_s {r['delivered_lines_per_blast_s']/1e6:6.2f} "
          f"fraction {r['delivered_fraction']:.3f} head {r['sink_head_s']} tail {r['sink_tail_s']}")
PY
