#!/bin/bash
# C4 emulated on one GPU (8 x 1M-lane replicas, 16 slices): exchange variants, 4 seeds, the
# exploitability after 1..4 steps (8.4M .. 33.5M total hands).  Output: gpurun_out/c4x_*.json
set -e
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 300 python3 -u tests/studies/exploit_group.py --replicas 8 --lanes 8388608 --every 8388608 \
    --hands ${HANDS:-33554432} --seeds ${SEEDS:-4} --slices 16 "$@" > gpurun_out/c4x_$name.json
  python3 - gpurun_out/c4x_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
b = d["bands"]["gpu_r8"]
print(sys.argv[2], {int(h) // 1000000: (round(m, 3), round(s, 3)) for h, (m, s) in b.items()},
      "rate", [round(r["hands_per_s_incl_eval"] / 1e6, 1) for r in d["gpu"]["8"]["rates"]],
      "frozen", d["gpu"]["8"]["frozen_seeds"], flush=True)
PY
}
for v in "$@"; do
  case $v in
    step_lag1) run $v ;;
    slice_ar_mean) run $v --slice-lag 2 --xchg-every 1 ;;
    slice_ar_sum) run $v --slice-lag 2 --xchg-every 1 --xchg-scale sum ;;
    slice_arbr_mean) run $v --slice-lag 2 --xchg-every 1 --xchg-nets arbr ;;
    slice_arbr_sum) run $v --slice-lag 2 --xchg-every 1 --xchg-nets arbr --xchg-scale sum ;;
    step_lag2) run $v --slice-lag 2 ;;
    ar_s*) run $v --slice-lag 2 --xchg-every 1 --xchg-scale ${v#ar_s} ;;
    arbr_s*) run $v --slice-lag 2 --xchg-every 1 --xchg-nets arbr --xchg-scale ${v#arbr_s} ;;
    k32_ar_g*) run $v --slices 32 --slice-lag 2 --xchg-every 1 --xchg-scale $(python3 -c "print(${v#k32_ar_g} / 8)") ;;
    k16_ar_g*) run $v --slices 16 --slice-lag 2 --xchg-every 1 --xchg-scale $(python3 -c "print(${v#k16_ar_g} / 8)") ;;
    k64_ar_g*) run $v --slices 64 --slice-lag 2 --xchg-every 1 --xchg-scale $(python3 -c "print(${v#k64_ar_g} / 8)") ;;
    k128_ar_g*) run $v --slices 128 --slice-lag 2 --xchg-every 1 --xchg-scale $(python3 -c "print(${v#k128_ar_g} / 8)") ;;
    k32_ar_s*) run $v --slices 32 --slice-lag 2 --xchg-every 1 --xchg-scale ${v#k32_ar_s} ;;
    k64_ar_s*) run $v --slices 64 --slice-lag 2 --xchg-every 1 --xchg-scale ${v#k64_ar_s} ;;
    k64_arbr_s*) run $v --slices 64 --slice-lag 2 --xchg-every 1 --xchg-nets arbr --xchg-scale ${v#k64_arbr_s} ;;
  esac
done
