#!/bin/bash
# Textbook NFSP on Kuhn (C5) at small lane counts, several settings side by side on one GPU
# (one process each, run concurrently): exploitability curves -> gpurun_out/kuhn_<tag>.jsonl.
#   tools/kuhn_sweep.sh <hands>
H=${1:-40000000}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
run() {   # tag lanes quirks rl sl [--set k=v ...]
  tag=$1; lanes=$2; q=$3; rl=$4; sl=$5; shift 5
  steps=$((H / lanes)); every=$((steps / 40))
  timeout -k 10 900 python tools/exploit_curve.py --config custom --lanes $lanes --game kuhn --quirks $q \
    --rl-capacity $rl --sl-capacity $sl --steps $steps --every $every "$@" > $O/kuhn_$tag.jsonl 2> $O/kuhn_$tag.err
  echo "$tag rc=$? $(tail -1 $O/kuhn_$tag.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["hands"], round(d["exploitability_softmax"],3))')"
}
run ref256 256 7 200000 2000000 &
run tb256 256 248 200000 2000000 &
run tb256lr 256 248 200000 2000000 --set lr_ar=0.005 --set lr_br=0.1 --set gamma=1.0 &
run tb1024lr 1024 248 200000 2000000 --set lr_ar=0.005 --set lr_br=0.1 --set gamma=1.0 &
run tb256lrs 256 248 20000 200000 --set lr_ar=0.005 --set lr_br=0.1 --set gamma=1.0 &
run tb256lr120 256 120 200000 2000000 --set lr_ar=0.005 --set lr_br=0.1 --set gamma=1.0 &
wait
