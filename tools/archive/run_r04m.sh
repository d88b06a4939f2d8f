#!/bin/bash
# which packed chain breaks the CU-sharing group test (R = 200)?
B=tools/bin
steps=()
for v in nopk brpk arpk brw brl2o; do steps+=("150 NFSP_LIB=$B/libnfsp_$v.so python3 -u tools/group_share_probe.py 200 2"); done
steps+=("150 python3 -u tools/group_share_probe.py 200 2")
./tools/gpu_steps.sh "${steps[@]}"
