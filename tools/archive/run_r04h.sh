#!/bin/bash
# the exact-order DPP backward + unrolled chain: GPU suite, smoke, the driver's bench command
./tools/gpu_steps.sh \
 "900 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gputest_ex.txt 2>&1; tail -3 gpurun_out/r04_gputest_ex.txt" \
 "300 python3 -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_ex.json"
