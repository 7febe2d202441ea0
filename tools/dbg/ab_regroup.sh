# Same-box A/B of the regroup leg: working tree vs tools/dbg/old/{regroup.py,bench.py}
set -e
mkdir -p gpurun_out/ab /tmp/abold
out=gpurun_out/ab/regroup.jsonl
: > $out
tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -C /tmp/abold -xf -
cp tools/dbg/old/regroup.py /tmp/abold/statsd-router_amd/regroup.py
cp tools/dbg/old/bench.py /tmp/abold/bench.py
for rep in 1 2; do
  r=$(timeout -k 10 120 python bench.py --regroup on --regroup-steps 64 --no-cpu --no-e2e --steps 256 --warmup 64 2>/dev/null); echo "new $r" >> $out
  r=$(cd /tmp/abold && timeout -k 10 120 python bench.py --regroup on --regroup-steps 64 --no-cpu --no-e2e --steps 256 --warmup 64 2>/dev/null); echo "old $r" >> $out
done
