#!/bin/bash
# round 5 (session 3): the persistent group BR kernel on the GPU -- a tiny group with short
# bounded waits, then the group / exchange suites with it, then c4_emul_r8 / c3_r16 timelines
# with it and with the rounds.  Ran at commit 8be66af: step 1 hung (profiles/r05_group_br_persist/),
# and the kernel and tools/brp_debug.py were removed after it.
./tools/gpu_steps.sh \
 "90 NFSP_GROUP_BR_PERSIST=1 NFSP_BRP_DEBUG=1 python3 -u tools/brp_debug.py 2 3" \
 "90 NFSP_GROUP_BR_PERSIST=1 NFSP_BRP_DEBUG=1 python3 -u tools/brp_debug.py 8 2 40" \
 "600 NFSP_GROUP_BR_PERSIST=1 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py -x -v --timeout 300 --timeout-method thread" \
 "200 NFSP_GROUP_BR_PERSIST=1 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_persist_c4emul.json" \
 "200 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_rounds_c4emul.json" \
 "200 NFSP_GROUP_BR_PERSIST=1 python3 -u tools/group_timeline.py c3_r16 3 6 > gpurun_out/r05_tl_persist_c3_r16.json" \
 "200 python3 -u tools/group_timeline.py c3_r16 3 6 > gpurun_out/r05_tl_rounds_c3_r16.json"
