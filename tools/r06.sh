#!/bin/bash
# Round 6's GPU jobs, one parameterised script (tools/gpu_steps.sh runs each step under its own
# time limit and stops after a fault or a timeout).   gpurun -- ./tools/r06.sh <job>
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
PYT="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
case "$1" in
  sched_kuhn)   # the group schedule test + C5 to 400M+ hands (item 6)
    ./tools/gpu_steps.sh \
      "400 $PYT tests/test_gpu_group.py tests/test_gpu_exchange.py -m gpu > $O/pytest_group.log" \
      "300 python3 -u tools/exploit_curve.py --config c5 --quirks 504 --set slices=16 --set slice_lag=2 --steps 420 --every 20 > $O/kuhn_tb_slices16.jsonl" \
      "300 python3 -u tools/exploit_curve.py --config c5 --set slices=16 --set slice_lag=2 --steps 420 --every 42 > $O/kuhn_ref_slices16.jsonl"
    ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
