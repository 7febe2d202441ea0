# product vs the previous library (C2, C4), and the opt-in mixed-lanes variant on C5 with its
# parity suite (SR_VARIANT is read once per process by the library)
set -e
CONFIGS="c2 c4" REPS=2 bash tools/dbg/ab_cfg.sh
SR_VARIANT=mixed_lanes timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_mixed.log 2>&1
for rep in 1 2; do
  r=$(SR_VARIANT=mixed_lanes timeout -k 10 120 python bench.py --config c5 --no-cpu --no-e2e 2>/dev/null); echo "c5 mixed $r" >> gpurun_out/ab/old.jsonl
  r=$(timeout -k 10 120 python bench.py --config c5 --no-cpu --no-e2e 2>/dev/null); echo "c5 product $r" >> gpurun_out/ab/old.jsonl
done
