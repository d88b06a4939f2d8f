#!/bin/bash
# round 5 (session 3): BR partitions on their own streams for sliced groups (default 2), each
# call's partitions after the previous call's BR snapshot -- the group / exchange / slices
# suites (bit-identity with standalone engines, the C4 gate), then c4_emul_r8 timelines with
# 1 / 2 / 3 BR streams and c3_r16 with 1 / 2 (partitions take their own BR results and snapshots)
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py tests/test_gpu_slices.py -x -v --timeout 400 --timeout-method thread" \
 "200 NFSP_GROUP_BR_STREAMS=1 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_brs1.json" \
 "200 NFSP_GROUP_BR_STREAMS=2 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_brs2.json" \
 "200 NFSP_GROUP_BR_STREAMS=3 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_brs3.json" \
 "200 NFSP_GROUP_BR_STREAMS=1 python3 -u tools/group_timeline.py c3_r16 3 6 > gpurun_out/r05_tl_c3r16_brs1.json" \
 "200 NFSP_GROUP_BR_STREAMS=2 python3 -u tools/group_timeline.py c3_r16 3 6 > gpurun_out/r05_tl_c3r16_brs2.json"
