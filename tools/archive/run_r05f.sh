#!/bin/bash
# round 5: capped BR rounds for the unsliced groups (c3_r16 / c3_r64 / c3_r256)
args=()
for cfg in c3_r16 c3_r64 c3_r256; do
  for cap in 0 40 100; do
    args+=("120 NFSP_GROUP_BR_CAP=$cap python3 -u tools/group_timeline.py $cfg 5 10 > gpurun_out/r05_tl_${cfg}_cap$cap.json")
  done
done
./tools/gpu_steps.sh "${args[@]}"
