#!/bin/bash
# round 5: C4 at 128 slices -- the learning gate, the rank-path equivalence tests, and the
# per-rank world-1 line with the RCCL exchange beside C3
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_slices.py::test_c4_emulated_learns_within_the_cpu_seed_band tests/test_gpu_exchange.py tests/test_gpu_group.py -x -v -s --timeout 500 --timeout-method thread" \
 "300 python3 -u bench.py --config c4 --ar-allreduce on --steps 10 --warmup 3 --no-cpu --groups '' > gpurun_out/r05_c4_rank_xchg_world1.json" \
 "300 python3 -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu --groups '' > gpurun_out/r05_c3_nocpu.json"
