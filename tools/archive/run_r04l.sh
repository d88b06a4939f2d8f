#!/bin/bash
# round 4, packed f32 in the SGD chains: the microbenchmark A/B against the scalar chain
# (weight hashes), the GPU suite, and bench.py with the driver's command
./tools/gpu_steps.sh \
 "120 ./tools/ar_var.sh 3 base fin -- base fin" \
 "700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_pk.json"
