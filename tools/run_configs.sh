#!/bin/bash
# bench.py lines for the other BASELINE configs on one box: tools/run_configs.sh <tag> cfg...
set -o pipefail
tag=${1:?tag}; shift
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $O
for c in "$@"; do
  timeout -k 10 400 python bench.py --config $c --groups '' --steps ${STEPS:-10} --warmup ${WARMUP:-3} > $O/${tag}_$c.json 2> $O/${tag}_$c.err || { tail -20 $O/${tag}_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/${tag}_$c.json')); print('$c', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', 'ins/hand', round(d['per_step']['rl_inserts_per_hand'],2), 'expl', round(d['exploitability_exact']['softmax_mixed'],3), 'cpu', round(d.get('cpu_baseline',{}).get('value',0)/1e6,3))"
done
