#!/bin/bash
# Same-box A/B of library builds over bench.py argument sets, alternating build by build, round by round:
#   bash tools/ab_bench.sh <out.jsonl> <rounds> <lib dir>[,<lib dir>...] "<bench args>" ["<bench args>" ...]
# A lib dir holds libsr_route.so ("-" = the in-tree build). Every bench line is appended to out.jsonl with
# {"ab_lib": dir, "ab_args": args}; python tools/ab_summary.py <out.jsonl> tabulates them.
out=$1; rounds=$2; libs=$3; shift 3
mkdir -p "$(dirname "$out")"
for r in $(seq 1 "$rounds"); do
  for a in "$@"; do
    for d in ${libs//,/ }; do
      lib=""; [ "$d" != "-" ] && lib="$d/libsr_route.so"
      line=$(SR_ROUTE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-e2e $a 2>"$out.err") || { tail -20 "$out.err"; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); d['ab_lib']=sys.argv[2]; d['ab_args']=sys.argv[3]; d['ab_round']=int(sys.argv[4]); print(json.dumps(d))" "$line" "$d" "$a" "$r" >> "$out"
      echo "round $r lib $d args $a done"
    done
  done
done
