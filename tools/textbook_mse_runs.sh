#!/bin/bash
# Textbook NFSP with the MSE Q loss (quirks 504) on Kuhn (C5) and Leduc, side by side on one GPU
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
c() { tag=$1; shift; timeout -k 10 900 python tools/exploit_curve.py --config custom --rl-capacity 200000 --sl-capacity 2000000 "$@" > $O/tm_$tag.jsonl 2> $O/tm_$tag.err; echo "$tag rc=$?"; }
c kuhn_c5 --game kuhn --lanes 1048576 --quirks 504 --steps 60 --every 5 &
c kuhn_r64 --game kuhn --lanes 16384 --replicas 64 --quirks 504 --steps 60 --every 5 &
c leduc16k_504 --lanes 16384 --quirks 504 --steps 2000 --every 200 &
c leduc16k_ref --lanes 16384 --quirks 7 --steps 2000 --every 200 &
c leduc_r16_504 --lanes 65536 --replicas 16 --quirks 504 --steps 32 --every 2 &
c leduc_r64_504 --lanes 16384 --replicas 64 --quirks 504 --steps 64 --every 4 &
wait
