set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread -k "slices and not learns_within" > $O/pytest_gpu_r03b.log 2>&1 || { tail -40 $O/pytest_gpu_r03b.log; exit 1; }
tail -3 $O/pytest_gpu_r03b.log
for c in c3 c3_1slice; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --groups '' --steps 10 --warmup 3 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', {x: round(v,2) for x,v in d['kernel_ms_per_step'].items()}, 'ins/hand', round(d['per_step']['rl_inserts_per_hand'],2), 'expl', round(d['exploitability_exact']['softmax_mixed'],3))"
done
