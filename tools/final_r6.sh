#!/bin/bash
# Round-6 final pass on one box, on the shipped build only. Steps (default: all, in this order; pmc
# first so that the bench lines after it report this library's HBM traffic):
#   tests   every -m gpu test, then __graft_entry__.smoke()
#   bench   the default bench command three times; C2..C5 lines, all alive and 25 % dead, with route + pack
#           and two data threads
#   regroup the regroup leg on one GPU (sr_regroup_launch, two contexts alternating; C5 also one context)
#   prof    rocprofv3 kernel stats (CSV) of the C2 and C5 commands and of the C5 regroup leg
#   pmc     PMC passes of the C2 command (bench_traffic.json for this library) and of the C5 command
#   c1      config C1 over loopback: this router and the reference executable, 10 s blasts
# Everything goes under gpurun_out/$T/ (T defaults to fin6).
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${FIN_TAG:-fin6}
O=gpurun_out/$T
cd "$R" || exit 1
mkdir -p "$O"
export TMPDIR=/tmp
steps=${*:-"pmc tests bench regroup prof c1"}
b() {   # b <name> <bench args...>: one bench line into $O/<name>.json
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$O/$name.json" 2> "$O/$name.err" || { tail -20 "$O/$name.err"; exit 1; }
  echo "$name done"
}
for st in $steps; do
  case $st in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
      || { tail -30 "$O/gpu_tests.log"; exit 1; }
    tail -1 "$O/gpu_tests.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
    cat "$O/smoke.log" ;;
  bench)
    for k in 1 2 3; do b bench_default_run$k; done
    for c in c2 c3 c4 c5; do
      for dead in 0 0.25; do b bench_${c}_dead$dead --config $c --dead $dead --no-cpu --no-e2e --pack-threads 2; done
    done ;;
  regroup)
    for c in c5 c2 c3; do b regroup_${c}_slots2 --config $c --steps 20 --no-cpu --no-e2e --no-pack --regroup on --regroup-config $c --regroup-steps 24; done
    b regroup_c5_slots1 --config c5 --steps 20 --no-cpu --no-e2e --no-pack --regroup on --regroup-config c5 --regroup-steps 24 --regroup-slots 1 ;;
  prof)
    for job in "c2|--config c2" "c5|--config c5" "c3_dead|--config c3 --dead 0.25" \
               "c5_regroup|--config c5 --steps 20 --no-pack --regroup on --regroup-steps 24"; do
      name=${job%%|*}; args=${job#*|}
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_$name" -o run \
         -- python "$R/bench.py" $args --no-cpu --no-e2e > "$R/$O/prof_$name.json" 2> "$R/$O/prof_$name.err") \
        || { tail -20 "$O/prof_$name.err"; exit 1; }
      echo "prof $name done"
    done ;;
  pmc)
    bash tools/pmc_passes.sh "$O/pmc_c2" --config c2 --steps 100 --no-pack || exit 1
    python tools/pmc_summary.py "$O/pmc_c2" c2 "$O/pmc_summary_c2.json" "$O/bench_traffic_c2.json" --kernel route_kernel || exit 1
    cp "$O/bench_traffic_c2.json" bench_traffic.json   # this box's copy: the bench steps after it report the traffic
    bash tools/pmc_passes.sh "$O/pmc_c5" --config c5 --steps 100 --no-pack || exit 1
    python tools/pmc_summary.py "$O/pmc_c5" c5 "$O/pmc_summary_c5.json" "$O/bench_traffic_c5.json" --kernel route_chunk_kernel || exit 1 ;;
  c1)
    timeout -k 10 600 python tools/loopback/c1_bench.py --seconds 10 > "$O/c1_loopback_10s.jsonl" 2> "$O/c1.err" \
      || { tail -20 "$O/c1.err"; exit 1; } ;;
  esac
done
