#!/bin/bash
# round 5: the persistent group BR kernel -- parity suites (groups of <= 32 replicas take it),
# then c4_emul_r8 / c3_r16 / c3_r4 with it and with the rounds (NFSP_GROUP_BR_PERSIST=0)
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py tests/test_gpu_slices.py -x -v -s --timeout 500 --timeout-method thread" \
 "200 python3 -u tools/group_timeline.py c4_emul_r8 1 2 > gpurun_out/r05_tl_persist_c4emul.json" \
 "200 NFSP_GROUP_BR_PERSIST=0 python3 -u tools/group_timeline.py c4_emul_r8 1 2 > gpurun_out/r05_tl_rounds_c4emul.json" \
 "200 python3 -u tools/group_timeline.py c3_r16 5 10 > gpurun_out/r05_tl_persist_c3_r16.json" \
 "200 NFSP_GROUP_BR_PERSIST=0 python3 -u tools/group_timeline.py c3_r16 5 10 > gpurun_out/r05_tl_rounds_c3_r16.json" \
 "200 python3 -u tools/group_timeline.py c3_r4 5 10 > gpurun_out/r05_tl_persist_c3_r4.json" \
 "200 NFSP_GROUP_BR_PERSIST=0 python3 -u tools/group_timeline.py c3_r4 5 10 > gpurun_out/r05_tl_rounds_c3_r4.json"
