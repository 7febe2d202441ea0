#!/bin/bash
# PMC passes of the default bench command's dominant kernel (one rocprofv3 --pmc run per counter
# group, never combined with tracing), summarised into gpurun_out/<tag>_pmc_summary_<cfg>.json and the
# traffic record gpurun_out/<tag>_bench_traffic_<cfg>.json (copied to ./bench_traffic.json when the
# library it names is the one shipped).
# Usage: bash tools/r4_pmc.sh <tag> [config] [bench args...]
tag=${1:-r4}; cfg=${2:-c2}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_pmc_$cfg
rm -rf "$out"
bash tools/pmc_passes.sh "$out" --config "$cfg" --steps 30 --warmup 5 --no-pack --regroup off "$@" || exit 1
python tools/pmc_summary.py "$out" "$cfg" gpurun_out/${tag}_pmc_summary_$cfg.json gpurun_out/${tag}_bench_traffic_$cfg.json > /dev/null || exit 1
python - "$tag" "$cfg" <<'PY'
import json, sys
tag, cfg = sys.argv[1:3]
d = json.load(open(f"gpurun_out/{tag}_pmc_summary_{cfg}.json"))
m = d["median_per_dispatch"]
w = m.get("SQ_WAVES", 0) or 1
print(cfg, d["kernel"], "dispatches", d["dispatches"], "read MB", round(d.get("hbm_read_bytes_per_launch", 0) / 1e6, 1),
      "write MB", round(d.get("hbm_write_bytes_per_launch", 0) / 1e6, 1),
      "VALU/wave", round(m.get("SQ_INSTS_VALU", 0) / w, 1), "SALU/wave", round(m.get("SQ_INSTS_SALU", 0) / w, 1),
      "LDS/wave", round(m.get("SQ_INSTS_LDS", 0) / w, 1), "meta", d.get("kernel_meta"))
PY
