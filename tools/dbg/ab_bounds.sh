set -e
mkdir -p gpurun_out/ab
out=gpurun_out/ab/bounds.jsonl
: > $out
for rep in 1 2; do
  for c in ${CONFIGS:-c2 c4}; do
    for v in default fake_base no_hash fake_base_no_hash no_lines; do
      vv=$v; [ "$v" = default ] && vv=""
      r=$(SR_VARIANT=$vv timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --steps 1024 2>/dev/null)
      echo "$c $v 16 $r" >> $out
    done
  done
done
