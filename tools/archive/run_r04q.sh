#!/bin/bash
# round 4 final tree: the GPU suite, smoke(), the driver's bench command, and the 2-rank
# co-resident gloo rehearsal of the C4 rank path (bench.py --gpus 2 on one GPU)
./tools/gpu_steps.sh \
 "700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "300 python3 -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_final_pk.json" \
 "600 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu --groups '' > gpurun_out/r04_c4_x2_gloo_pk.json"
