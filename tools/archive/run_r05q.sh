#!/bin/bash
# round 5 (session 3): paced BR pieces at caps 30 / 50 / 64 / 80 (2 partitions)
./tools/gpu_steps.sh \
 "200 NFSP_GROUP_BR_CAP=30 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_paced_cap30.json" \
 "200 NFSP_GROUP_BR_CAP=50 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_paced_cap50.json" \
 "200 NFSP_GROUP_BR_CAP=64 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_paced_cap64.json" \
 "200 NFSP_GROUP_BR_CAP=80 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_paced_cap80.json"
