#!/bin/bash
# One GPU call: the -m gpu suite (optionally a -k filter), then bench.py for each config.
#   tools/gpu_check.sh "<pytest -k expr or ALL or NONE>" cfg1 cfg2 ...
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
k=${1:-ALL}; shift
if [ "$k" != "NONE" ]; then
  if [ "$k" = "ALL" ]; then sel=(); else sel=(-k "$k"); fi
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${sel[@]}" > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps ${STEPS:-5} --warmup ${WARMUP:-2} > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); k=d['kernel_ms_per_step']; print('$c', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],2), 'ms', {x: round(v,3) for x,v in k.items()}, 'ins/hand', round(d['per_step']['rl_inserts_per_hand'],2), 'expl', round(d['exploitability_exact']['softmax_mixed'],3))"
done
