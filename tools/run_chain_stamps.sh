#!/bin/bash
# phase cycles of the final chain (diagnostic stamps build: s_memtime + lgkmcnt drain per phase)
B=${GRAFT_REPO_ROOT:-$(pwd)}/tools/bin
timeout -k 5 60 $B/bench_chain_stamps_br 400 1 time 1 && timeout -k 5 60 $B/bench_chain_stamps_ar 400 0 time 2
