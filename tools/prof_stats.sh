#!/bin/bash
# rocprofv3 kernel-trace stats of one bench.py command: tools/prof_stats.sh <tag> [bench args...]
# -> gpurun_out/prof_<tag>/ (CSV) and gpurun_out/prof_<tag>.txt (per-kernel mean us, calls)
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run \
    -- python "$R/bench.py" "$@" > "$R/gpurun_out/prof_$tag.json" 2> "$R/gpurun_out/prof_$tag.err" || exit 1
cd "$R" && python - "$tag" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
for f in glob.glob(f"gpurun_out/prof_{tag}/**/*kernel_stats.csv", recursive=True):
    with open(f) as fh, open(f"gpurun_out/prof_{tag}.txt", "w") as out:
        for row in csv.DictReader(fh):
            line = f"{row['Name'][:70]:70s} calls {row['Calls']:>6s} mean_us {float(row['AverageNs'])/1e3:9.2f} total_pct {float(row['Percentage']):6.2f}"
            print(line); out.write(line + "\n")
PY
