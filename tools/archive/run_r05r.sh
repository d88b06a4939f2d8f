#!/bin/bash
# round 5 (session 3): paced BR rounds with 2 / 3 / 4 halves, the timeline tool with 8 hardware queues
./tools/gpu_steps.sh \
 "200 NFSP_GROUP_BR_STREAMS=3 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_q8_brs3.json" \
 "200 NFSP_GROUP_BR_STREAMS=4 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_q8_brs4.json" \
 "200 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_q8_brs2.json"
