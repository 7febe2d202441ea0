# Same-box A/B (working tree vs tools/dbg/old/libsr_route.so) over CONFIGS, REPS repetitions
set -e
mkdir -p gpurun_out/ab /tmp/abold
out=gpurun_out/ab/old.jsonl
: > $out
tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -C /tmp/abold -xf -
cp tools/dbg/old/libsr_route.so /tmp/abold/statsd-router_amd/lib/libsr_route.so
for rep in $(seq ${REPS:-2}); do
  for c in ${CONFIGS:-c2 c5}; do
    r=$(timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e 2>/dev/null); echo "$c new $r" >> $out
    r=$(cd /tmp/abold && timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e 2>/dev/null); echo "$c old $r" >> $out
  done
done
