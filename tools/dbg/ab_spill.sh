set -e
mkdir -p gpurun_out/ab
for c in c2 c3 c4 c5; do
  timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps 1024 > gpurun_out/ab/spill_$c.json 2>/dev/null
  SR_SPILL=0 timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps 1024 > gpurun_out/ab/nospill_$c.json 2>/dev/null
  timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps 1024 > gpurun_out/ab/spill2_$c.json 2>/dev/null
done
