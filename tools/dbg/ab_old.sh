# Same-box A/B: the working-tree library vs tools/dbg/old/libsr_route.so (a previous build),
# bench.py from a copy of the tree with the library swapped. Lines appended to gpurun_out/ab/old.jsonl.
set -e
mkdir -p gpurun_out/ab /tmp/abold
out=gpurun_out/ab/old.jsonl
: > $out
tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -C /tmp/abold -xf -
cp tools/dbg/old/libsr_route.so /tmp/abold/statsd-router_amd/lib/libsr_route.so
for rep in $(seq ${REPS:-2}); do
  for c in ${CONFIGS:-c2 c4}; do
    r=$(timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps ${STEPS:-1024} 2>/dev/null); echo "$c new $r" >> $out
    r=$(cd /tmp/abold && timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps ${STEPS:-1024} 2>/dev/null); echo "$c old $r" >> $out
  done
done
