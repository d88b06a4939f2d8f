#!/bin/bash
# round 5 (session 3): background targets for the non-busiest jobs of each BR partition --
# the group / exchange / slices suites, then c4_emul_r8 with and without them
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py tests/test_gpu_slices.py -x -v --timeout 400 --timeout-method thread" \
 "200 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_bg.json" \
 "200 NFSP_GROUP_BR_BG=0 python3 -u tools/group_timeline.py c4_emul_r8 1 3 > gpurun_out/r05_tl_nobg.json"
