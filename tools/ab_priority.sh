for r in 1 2; do
for p in 0 -1; do
  for c in c2 c5; do
    out=$(timeout -k 10 120 python bench.py --config $c --no-cpu --no-e2e --no-verify --regroup off --steps 50 --second-priority $p 2>gpurun_out/ab_last.err) || { cat gpurun_out/ab_last.err; exit 1; }
    python -c "import json,sys; d=json.loads(sys.argv[1]); rp=d['route_pack']; print('prio', sys.argv[2], sys.argv[3], 'route_pack_ms', rp['ms_per_launch'], 'two', rp['two_threads']['ms_per_round'], rp['two_threads']['value'])" "$out" "$p" "$c"
  done
done
done
