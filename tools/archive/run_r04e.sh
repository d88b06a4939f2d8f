#!/bin/bash
# final-tree GPU suite, smoke, and the 2-rank co-resident rehearsal of the C4 rank path (gloo)
./tools/gpu_steps.sh \
 "900 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gputest.txt 2>&1; tail -3 gpurun_out/r04_gputest.txt" \
 "300 python3 -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r04_c4_x2_coresident_gloo.json"
