set -e
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
for c in c3 c4 c5; do timeout -k 10 200 python bench.py --config $c --no-e2e --cpu-seconds 1.0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err; done
timeout -k 10 200 python bench.py --config c2 --dead 0.25 --no-e2e --no-cpu > gpurun_out/bench_c2_dead.json 2> gpurun_out/bench_c2_dead.err
