#!/bin/bash
# Interleaved A/B of chain microbenchmark builds on one box (run through gpurun):
#   tools/chain_ab.sh <rounds> <tag> [<tag> ...]
# Each tag names tools/bin/bench_chain_<tag>_{ar,br} (tools/build_chain_bench.sh <tag> [flags]).
# Per round and tag: the BR chain (relu 1, one block) and the AR chain (relu 0, two blocks,
# as the engine launches it), 400 updates each; then "compare" of each build against the
# f32 reference chain.
set -o pipefail
n=${1:?rounds}; shift
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/bin
for i in $(seq $n); do
  for t in "$@"; do
    timeout -k 5 60 $B/bench_chain_${t}_br 400 1 time 1 | head -1 | sed "s/^/$t br: /" || exit 1
    timeout -k 5 60 $B/bench_chain_${t}_ar 400 0 time 2 | head -1 | sed "s/^/$t ar: /" || exit 1
  done
done
for t in "$@"; do
  timeout -k 5 60 $B/bench_chain_${t}_br 200 1 compare | sed "s/^/$t /"
  timeout -k 5 60 $B/bench_chain_${t}_ar 200 0 compare | sed "s/^/$t /"
done
exit 0
