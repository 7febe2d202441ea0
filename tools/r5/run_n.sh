#!/bin/bash
# Instruction counts of the chunk kernel, C5 all alive against 16 of 64 dead (one PMC group per run)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
for d in 0 0.25; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -c1-12 | tr ' ' '_')
    timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $O/r5n_pmc_${d}_$tag -o pmc -- python bench.py --config c5 --dead $d --no-cpu --no-e2e --no-pack --regroup off --steps 20 --warmup 3 > $O/r5n_pmc_${d}_$tag.log 2>&1 || { tail -20 $O/r5n_pmc_${d}_$tag.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, collections, statistics
for d in ("0", "0.25"):
    per = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/r5n_pmc_{d}_*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "route_chunk_kernel" in k or "probe_defer" in k:
                name = "chunk" if "chunk" in k else "defer"
                per[(name, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    vals = collections.defaultdict(list)
    for (n, _, c), v in per.items(): vals[(n, c)].append(v)
    for n in ("chunk", "defer"):
        m = {c: statistics.median(v) for (nn, c), v in vals.items() if nn == n}
        if not m: continue
        w = m.get("SQ_WAVES", 1) or 1
        print(d, n, {c: round(v / w, 1) for c, v in sorted(m.items()) if c.startswith("SQ_INSTS")}, "waves", m.get("SQ_WAVES"),
              {c: m[c] for c in ("SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE") if c in m})
PY
R=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/r5n_prof_c5dead" -o run \
   -- python "$R/bench.py" --config c5 --dead 0.25 --no-cpu --no-e2e --regroup off --steps 30 --warmup 5 > "$R/$O/r5n_prof_c5dead.json" 2> "$R/$O/r5n_prof_c5dead.err") || exit 1
