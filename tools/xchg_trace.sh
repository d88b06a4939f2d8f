#!/bin/bash
# HIP runtime trace of C4's per-rank line at world 1, with and without the RCCL exchange:
# which runtime calls does the exchange add, and do any of them block the host?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/xtrace
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in noxchg xchg; do
  extra=""
  [ $v = xchg ] && extra="--ar-allreduce on --xchg-gain 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d "$O" -o $v -- \
    python3 "$R/bench.py" --config c4 --no-cpu --groups '' --steps 2 --warmup 1 $extra > "$O/$v.json" 2> "$O/$v.err" || { tail -20 "$O/$v.err"; exit 1; }
done
ls "$O"
