#!/bin/bash
# round 5 (session 3): paced BR pieces in capped groups -- the group / exchange / slices suites,
# then c4_emul_r8 paced / unpaced (2 BR partitions) and 1 partition paced
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py tests/test_gpu_slices.py -x -v --timeout 400 --timeout-method thread" \
 "200 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_paced.json" \
 "200 NFSP_GROUP_BR_PACE=0 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_unpaced.json" \
 "200 NFSP_GROUP_BR_STREAMS=1 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_paced_brs1.json"
