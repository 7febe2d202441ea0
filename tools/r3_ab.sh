#!/bin/bash
# Route-kernel part ablation (timing + PMC instruction counts, 64-byte lines, 32 batches per launch)
# and a route+pack A/B of lib dirs. Usage (via gpurun): bash tools/r3_ab.sh <tag> [lib dirs...]
tag=${1:-cur}; shift
mkdir -p gpurun_out
if [ -n "$R3_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $R3_TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
timeout -k 10 300 tools/ablate_route 64 quick > gpurun_out/abl_${tag}.json 2> gpurun_out/abl_${tag}.err || { cat gpurun_out/abl_${tag}.err; exit 1; }
cat gpurun_out/abl_${tag}.json
bash tools/pmc_ablate.sh gpurun_out/pmcabl_${tag} 64 quick || exit 1
python tools/pmc_ablate_summary.py gpurun_out/pmcabl_${tag} > gpurun_out/pmcabl_${tag}.json || exit 1
python -c "
import json; d=json.load(open('gpurun_out/pmcabl_${tag}.json'))
for k,v in d.items(): print(k, 'VALU', v.get('SQ_INSTS_VALU'), 'SALU', v.get('SQ_INSTS_SALU'), 'LDS', v.get('SQ_INSTS_LDS'), 'cyc', v.get('SQ_WAVE_CYCLES'), 'waitany', v.get('SQ_WAIT_ANY'), 'waitinst', v.get('SQ_WAIT_INST_ANY'), 'active', v.get('SQ_ACTIVE_INST_ANY'))
"
if [ $# -gt 0 ]; then
  AB_CFGS="c2 c5" bash tools/ab_pack.sh 2 "$@" > gpurun_out/ab_pack_${tag}.txt 2>&1 || { cat gpurun_out/ab_pack_${tag}.txt; exit 1; }
  sort -k1,2 gpurun_out/ab_pack_${tag}.txt | awk '{print $1, $2, "route", $6, "packing", $8}'
fi
