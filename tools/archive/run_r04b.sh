#!/bin/bash
# the whole GPU suite on this tree, then the default bench line, then the 2-rank co-resident
# rehearsal of the C4 rank path (gloo, host transport)
./tools/gpu_steps.sh \
 "900 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gputest.txt 2>&1; tail -5 gpurun_out/r04_gputest.txt" \
 "400 python3 -u bench.py > gpurun_out/r04_bench_default.json" \
 "400 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r04_c4_x2_coresident_gloo.json"
