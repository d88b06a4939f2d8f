#!/bin/bash
# AR-only interleaved A/B with compare: tools/chain_ab_ar.sh <rounds> <tag>...
set -o pipefail
n=${1:?rounds}; shift
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/bin
for i in $(seq $n); do
  for t in "$@"; do
    timeout -k 5 60 $B/bench_chain_${t}_ar 400 0 time 2 | head -1 | sed "s/^/$t ar: /" || exit 1
  done
done
for t in "$@"; do
  timeout -k 5 60 $B/bench_chain_${t}_ar 200 0 compare | sed "s/^/$t /"
  timeout -k 5 60 $B/bench_chain_${t}_ar 200 0 compare 1 60 | sed "s/^/$t saturated: /"
done
exit 0
