#!/bin/bash
# round 5: the whole GPU suite on this tree, then the driver's exact bench command
./tools/gpu_steps.sh \
 "700 python3 -u -m pytest tests -m gpu -v --durations=15 --timeout 300 --timeout-method thread" \
 "480 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_driver_cmd.json"
