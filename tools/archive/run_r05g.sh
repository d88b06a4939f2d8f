#!/bin/bash
# round 5, final tree: the whole GPU suite, smoke(), the driver's exact bench command
./tools/gpu_steps.sh \
 "700 python3 -u -m pytest tests -m gpu -v --durations=10 --timeout 300 --timeout-method thread" \
 "300 python3 -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "480 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_final.json"
