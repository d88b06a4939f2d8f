#!/bin/bash
# round 5 (session 3): the partition determinism test; c4_emul_r8 with 2 BR partitions at BR
# piece caps 24 / 64 / 100
./tools/gpu_steps.sh \
 "300 python3 -u -m pytest tests/test_gpu_group.py -k deterministic -x -v --timeout 250 --timeout-method thread" \
 "200 NFSP_GROUP_BR_CAP=24 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_brs2_cap24.json" \
 "200 NFSP_GROUP_BR_CAP=64 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_brs2_cap64.json" \
 "200 NFSP_GROUP_BR_CAP=100 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_brs2_cap100.json"
