#!/bin/bash
# rocprofv3 kernel stats of the default bench command for C2 and C5 (the route kernel's mean then
# matches the line), and the two-data-thread route + pack figures (bench.py --pack-threads 2).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c2 c5; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/fin2_prof_$c" -o run \
     -- python "$R/bench.py" --config $c --no-cpu --no-e2e > "$R/gpurun_out/fin2_prof_$c.json" 2> "$R/gpurun_out/fin2_prof_$c.err") || exit 1
done
for c in c2 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu --no-e2e --pack-threads 2 > gpurun_out/fin2_two_$c.json 2> gpurun_out/fin2_two_$c.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fin2_two_$c.json')); rp=d['route_pack']; print('$c', d['value'], d['roofline']['frac'], rp['value'], rp['packing_ms'], rp['two_threads']['value'], rp['two_threads']['ms_per_round'])"
done
for c in c2 c5; do
  python - "$c" <<'PY'
import csv, json, sys
c = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/fin2_prof_{c}/run_kernel_stats.csv")))
d = json.load(open(f"gpurun_out/fin2_prof_{c}.json"))
print(c, "line", d["value"], d["roofline"]["frac"], d["roofline"]["launch_us"])
for r in rows[:9]:
    print(c, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
