#!/bin/bash
# AR / BR variants of the chain microbenchmark, interleaved: tools/ar_var.sh <rounds> <ar tags> -- <br tags>
B=tools/bin
n=$1; shift
ar=(); br=(); cur=ar
for t in "$@"; do if [ "$t" = "--" ]; then cur=br; elif [ $cur = ar ]; then ar+=($t); else br+=($t); fi; done
for i in $(seq $n); do
  for t in "${ar[@]}"; do timeout -k 5 60 $B/bench_chain_${t}_ar 400 0 time 2 | head -1 | sed "s/^/$t ar: /" || exit 1; done
  for t in "${br[@]}"; do timeout -k 5 60 $B/bench_chain_${t}_br 400 1 time 1 | head -1 | sed "s/^/$t br: /" || exit 1; done
done
for t in "${ar[@]}"; do timeout -k 5 60 $B/bench_chain_${t}_ar 200 0 compare | sed "s/^/$t /" || exit 1; done
for t in "${br[@]}"; do timeout -k 5 60 $B/bench_chain_${t}_br 200 1 compare | sed "s/^/$t /" || exit 1; done
