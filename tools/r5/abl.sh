#!/bin/bash
# Same-box A/B of route-kernel builds and layouts plus per-variant instruction counts.
#   bash tools/r4_abl.sh <tag> <rounds> "<cfgs>" <variant>...
# variant = <name>@<lib dir or "cur">@<layout>. Timing: bench.py route-only launches (µs per 32-batch
# launch) alternating between variants; counts: one rocprofv3 --pmc pass (SQ_WAVES, SQ_INSTS_VALU,
# SQ_INSTS_SALU, SQ_INSTS_LDS) per variant on C2. Ablation builds write wrong records: --no-verify.
tag=$1; rounds=$2; cfgs=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.jsonl
: > $out
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    IFS=@ read -r name lib lay <<< "$v"
    libpath=$R/statsd-router_amd/lib/libsr_route.so
    [ "$lib" != "cur" ] && libpath=$R/$lib/libsr_route.so
    for c in $cfgs; do
      o=$(SR_ROUTE_LIB=$libpath timeout -k 10 120 python bench.py --config $c --layout $lay --no-cpu --no-e2e --no-verify \
          --no-pack --regroup off --steps 300 2> gpurun_out/${tag}_last.err) || { tail -20 gpurun_out/${tag}_last.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'v': sys.argv[2], 'cfg': sys.argv[3], 'launch_us': d['roofline']['launch_us'], 'frac': d['roofline']['frac']}))" "$o" "$name" "$c" >> $out
    done
  done
done
python - $out <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); agg[(r["cfg"], r["v"])].append(r["launch_us"])
for k in sorted(agg): print(k, ["%.1f" % x for x in agg[k]], "min %.1f" % min(agg[k]))
PY
export TMPDIR=/tmp
for v in "$@"; do
  IFS=@ read -r name lib lay <<< "$v"
  libpath=$R/statsd-router_amd/lib/libsr_route.so
  [ "$lib" != "cur" ] && libpath=$R/$lib/libsr_route.so
  d=gpurun_out/${tag}_pmc_$name
  rm -rf $d
  SR_ROUTE_LIB=$libpath timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv \
      -d $d -o pmc -- python bench.py --config ${PMC_CFG:-c2} --layout $lay --no-cpu --no-e2e --no-verify --no-pack --regroup off \
      --steps 20 --warmup 3 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python - $d $name <<'PY'
import csv, glob, sys, statistics, collections
d, name = sys.argv[1:3]
per = collections.defaultdict(float)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "route" in row["Kernel_Name"] and "kernel" in row["Kernel_Name"] and "probe" not in row["Kernel_Name"]:
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
vals = collections.defaultdict(list)
for (_, c), v in per.items(): vals[c].append(v)
m = {c: statistics.median(v) for c, v in vals.items()}
w = m.get("SQ_WAVES", 1) or 1
print(name, "VALU/wave %.1f SALU/wave %.1f LDS/wave %.1f" % (m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_SALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w))
PY
done
