set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread -k "slices or group" > $O/pytest_gpu_r03c.log 2>&1 || { tail -40 $O/pytest_gpu_r03c.log; exit 1; }
tail -3 $O/pytest_gpu_r03c.log
for v in "16 1" "16 2" "32 2" "64 2"; do set -- $v
  timeout -k 10 300 python bench.py --config c3 --slices $1 --slice-lag $2 --no-cpu --groups '' --steps 10 --warmup 3 > $O/bench_c3_$1_$2.json 2> $O/bench_c3_$1_$2.err || { tail -20 $O/bench_c3_$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_c3_$1_$2.json')); print('$1 $2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', {x: round(v,2) for x,v in d['kernel_ms_per_step'].items()}, 'ins/hand', round(d['per_step']['rl_inserts_per_hand'],2), 'expl', round(d['exploitability_exact']['softmax_mixed'],3))"
done
timeout -k 10 600 python -u tests/studies/exploit_slices.py --variants 16:1 16:2 32:2 > $O/exploit_slices.json 2> $O/exploit_slices.err || { tail -5 $O/exploit_slices.err; exit 1; }
python -c "
import json; d=json.load(open('$O/exploit_slices.json'))
cb=d['cpu_band']
for v,g in d['gpu'].items():
    print(v, [(int(h)//1000000, round(m,3), round(s,3)) for h,(m,s) in g['band'].items()])
print('cpu', [(int(h)//1000000, round(m,3), round(s,3)) for h,(m,s) in cb.items() if int(h) % 8000000 == 0])
"
