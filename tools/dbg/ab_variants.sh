# Same-box A/B of compiled-in kernel variants (SR_VARIANT) with bench.py; JSON lines appended to
# gpurun_out/ab/variants.jsonl as "<config> <variant> <json>".
set -e
mkdir -p gpurun_out/ab
out=gpurun_out/ab/variants.jsonl
: > $out
for rep in 1 2; do
  for c in ${CONFIGS:-c2 c4}; do
    for v in ${VARIANTS:-default agent_granules}; do
      vv=$v; [ "$v" = default ] && vv=""
      r=$(SR_VARIANT=$vv timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps 1024 2>/dev/null)
      echo "$c $v $r" >> $out
    done
  done
done
