#!/bin/bash
# Round-5 final pass on one box, this build only: every -m gpu test; the regroup leg (sr_regroup_launch, the same calls one by
# one, own chunk copied); the default bench line and
# C2..C5 lines (all alive and 25 % dead) with route + pack; rocprofv3 kernel stats of the default
# command for C2 and C5; the PMC traffic of the default command (copied to ./bench_traffic.json
# afterwards: it names the library it was measured with); C1 over loopback with 10 s blasts against round 2's data thread and the
# reference executable. Everything under gpurun_out/${T}_*.
# Usage: bash tools/r5_final.sh [steps...]   (default: tests bench prof pmc regroup c1)
R=${GRAFT_REPO_ROOT:-$(pwd)}
export T=${FIN_TAG:-fin5}   # output prefix under gpurun_out/
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
steps=${*:-"tests bench prof pmc regroup c1"}
for st in $steps; do
  case $st in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
    tail -1 gpurun_out/${T}_gpu_tests.log ;;
  bench)
    timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err \
      || { tail -20 gpurun_out/${T}_bench_default.err; exit 1; }
    for c in c2 c3 c4 c5; do
      for dead in 0 0.25; do
        timeout -k 10 300 python bench.py --config $c --dead $dead --no-cpu --no-e2e --pack-threads 2 \
          > gpurun_out/${T}_bench_${c}_dead$dead.json 2> gpurun_out/${T}_bench_${c}_dead$dead.err \
          || { tail -20 gpurun_out/${T}_bench_${c}_dead$dead.err; exit 1; }
      done
    done
    python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/" + os.environ["T"] + "_bench_*.json")):
    if "traffic" in f: continue
    d = json.load(open(f)); rp = d.get("route_pack") or {}
    print(f.split("/")[-1], d["value"], d["roofline"]["frac"], d["roofline"].get("launch_us"), d["config"].get("lane_layout"),
          "route+pack", rp.get("value"), rp.get("packing_ms"), "two", (rp.get("two_threads") or {}).get("value"),
          "traffic", d["roofline"].get("traffic"))
PY
    ;;
  prof)
    for c in c2 c5; do
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof_$c" -o run \
         -- python "$R/bench.py" --config $c --no-cpu --no-e2e > "$R/gpurun_out/${T}_prof_$c.json" 2> "$R/gpurun_out/${T}_prof_$c.err") || exit 1
      python - "$c" <<'PY'
import csv, json, sys
c = sys.argv[1]
T = __import__("os").environ["T"]
rows = list(csv.DictReader(open(f"gpurun_out/{T}_prof_{c}/run_kernel_stats.csv")))
d = json.load(open(f"gpurun_out/{T}_prof_{c}.json"))
print(c, "line", d["value"], d["roofline"]["frac"], d["roofline"]["launch_us"])
for r in rows[:10]:
    print(c, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
    done ;;
  pmc)
    bash tools/r4_pmc.sh $T c2 || exit 1 ;;   # gpurun_out/${T}_bench_traffic_c2.json -> ./bench_traffic.json here
  regroup)
    for c in c5 c2 c3; do
      for mode in inplace split copy; do
        extra=""; [ $mode = copy ] && extra="--regroup-copy-own"; [ $mode = split ] && extra="--regroup-split-calls"
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $c \
          --regroup-steps 32 $extra > gpurun_out/${T}_regroup_${c}_$mode.json 2> gpurun_out/${T}_regroup_${c}_$mode.err \
          || { tail -20 gpurun_out/${T}_regroup_${c}_$mode.err; exit 1; }
      done
    done
    python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/" + os.environ["T"] + "_regroup_*.json")):
    g = json.load(open(f))["regroup"]
    print(f.split("/")[-1], g.get("value"), g.get("ms_per_step"), g.get("error"))
PY
    ;;
  c1)
    bash tools/r4_c1_ab.sh $T 2 10 || exit 1 ;;
  esac
done
