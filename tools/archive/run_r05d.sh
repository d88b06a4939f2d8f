#!/bin/bash
# round 5: pipelined engine-group steps -- the group / exchange / C4-gate suites (bit-for-bit
# against pipelined ranks and standalone engines), then c4_emul_r8 pipelined vs serial
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py tests/test_gpu_slices.py -x -v -s --timeout 500 --timeout-method thread" \
 "300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu --groups c4_emul_r8 > gpurun_out/r05_c4emul_pipelined.json" \
 "300 NFSP_GROUP_SERIAL=1 python3 -u bench.py --steps 2 --warmup 1 --no-cpu --groups c4_emul_r8 > gpurun_out/r05_c4emul_serial.json"
