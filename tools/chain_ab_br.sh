#!/bin/bash
# BR-only (or AR-only with ar) interleaved A/B: tools/chain_ab_br.sh <rounds> <br|ar> <tag>...
set -o pipefail
n=${1:?rounds}; kind=${2:?br|ar}; shift 2
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/bin
for i in $(seq $n); do
  for t in "$@"; do
    if [ $kind = br ]; then timeout -k 5 60 $B/bench_chain_${t}_br 400 1 time 1 | head -1 | sed "s/^/$t br: /" || exit 1
    else timeout -k 5 60 $B/bench_chain_${t}_ar 400 0 time 2 | head -1 | sed "s/^/$t ar: /" || exit 1; fi
  done
done
exit 0
