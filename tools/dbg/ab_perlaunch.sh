set -e
mkdir -p gpurun_out/ab
out=gpurun_out/ab/perlaunch.jsonl
: > $out
for rep in 1 2; do
  for m in 16 32 8; do
    r=$(timeout -k 10 120 python bench.py --config c2 --no-cpu --no-e2e --per-launch $m 2>/dev/null); echo "c2 $m $r" >> $out
  done
done
