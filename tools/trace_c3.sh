#!/bin/bash
# Kernel trace of a short C3 bench run (rocprofv3 --kernel-trace, CSV) -> gpurun_out/trace/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O/trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o c3 -- \
  python3 "$R/bench.py" --config c3 --no-cpu --groups '' --steps ${STEPS:-3} --warmup ${WARMUP:-2} \
  > "$O/trace/bench.json" 2> "$O/trace/bench.err" || { tail -20 "$O/trace/bench.err"; exit 1; }
ls -la "$O/trace"
