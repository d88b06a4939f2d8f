#!/bin/bash
# round 5: capped BR rounds in engine groups -- parity suites, then c4_emul_r8 per cap
./tools/gpu_steps.sh \
 "600 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_exchange.py tests/test_gpu_slices.py -x -v -s --timeout 500 --timeout-method thread" \
 "200 NFSP_GROUP_BR_CAP=0 python3 -u tools/group_timeline.py c4_emul_r8 1 2 > gpurun_out/r05_tl_cap0.json" \
 "200 NFSP_GROUP_BR_CAP=40 python3 -u tools/group_timeline.py c4_emul_r8 1 2 > gpurun_out/r05_tl_cap40.json" \
 "200 NFSP_GROUP_BR_CAP=24 python3 -u tools/group_timeline.py c4_emul_r8 1 2 > gpurun_out/r05_tl_cap24.json" \
 "200 NFSP_GROUP_BR_CAP=64 python3 -u tools/group_timeline.py c4_emul_r8 1 2 > gpurun_out/r05_tl_cap64.json"
