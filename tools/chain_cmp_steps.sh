#!/bin/bash
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/bin
for u in 1 2 5 20 50 100 200 400; do
  for t in base dpp; do
    timeout -k 5 60 $B/bench_chain_${t}_ar $u 0 compare | sed "s/^/$t /" || exit 1
  done
done
for u in 1 5 50 200; do
  for t in base dpp; do
    timeout -k 5 60 $B/bench_chain_${t}_br $u 1 compare | sed "s/^/$t /" || exit 1
  done
done
