#!/bin/bash
# A/B of two trees on one box: tools/ab_bench.sh <config> <other tree> [rounds]
# Alternates `bench.py --config <config>` of this tree (new) and <other tree> (old).
set -o pipefail
cfg=${1:?config}; other=${2:?tree}; n=${3:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
for i in $(seq $n); do
  for t in new old; do
    d=$R; [ $t = old ] && d=$R/$other
    (cd $d && timeout -k 10 300 python bench.py --config $cfg --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/ab_${t}_$i.json 2> $R/gpurun_out/ab_${t}_$i.err) || { tail -5 $R/gpurun_out/ab_${t}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$R/gpurun_out/ab_${t}_$i.json')); k=d['kernel_ms']; print('$t', round(d['value']/1e6,3), round(d['ms_per_step'],2), 'br', round(k['k_chain3_br'],4), 'ar', round(k['k_chain3_ar'],2))"
  done
done
