#!/bin/bash
./tools/chain_ab.sh 3 ex tr1 tr2 || exit 1
B=tools/bin
timeout -k 5 60 $B/bench_chain_stamps_br 400 1 time 1
timeout -k 5 60 $B/bench_chain_stamps_ar 400 0 time 2
