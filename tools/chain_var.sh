#!/bin/bash
# Run-to-run spread of the chain microbenchmark: tools/chain_var.sh <tag> <runs>
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/bin
for i in $(seq ${2:-10}); do
  timeout -k 5 60 $B/bench_chain_${1}_br 400 1 time 1 | head -1 | sed "s/^/br1: /" || exit 1
  timeout -k 5 60 $B/bench_chain_${1}_br 400 1 time 2 | head -1 | sed "s/^/br2: /" || exit 1
done
exit 0
