#!/bin/bash
# round 5 (session 3), final tree (paced BR rounds): the whole GPU suite, smoke(), the driver's exact bench
# command, then rocprofv3 --kernel-trace --stats of that command and the two PMC passes
./tools/gpu_steps.sh \
 "700 python3 -u -m pytest tests -m gpu -v --durations=10 --timeout 300 --timeout-method thread" \
 "300 python3 -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "480 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_s3_final2.json" \
 "900 ./tools/run_r05c.sh"
