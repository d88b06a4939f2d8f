#!/bin/bash
# the deferred exchange: tests, C4 per-rank line with / without the world-1 exchange, trace gaps
./tools/gpu_steps.sh \
 "400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_exchange.py tests/test_gpu_slices.py -k 'exchange or declared or snapshot or pipelined'" \
 "300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 > gpurun_out/r04_c4_rank_noxchg.json" \
 "300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 --ar-allreduce on --xchg-gain 1 > gpurun_out/r04_c4_rank_xchg_world1.json" \
 "600 ./tools/xchg_trace.sh"
