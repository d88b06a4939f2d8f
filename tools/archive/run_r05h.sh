#!/bin/bash
# round 5: BR piece caps for unsliced groups at R = 32 / 64 / 128 (c3_r16 / c3_r256 measured in r05f)
args=()
for cfg in c3_r32 c3_r64 c3_r128; do
  for cap in 0 40 64; do
    args+=("120 NFSP_GROUP_BR_CAP=$cap python3 -u tools/group_timeline.py $cfg 5 10 > gpurun_out/r05_tl_${cfg}_cap$cap.json")
  done
done
./tools/gpu_steps.sh "${args[@]}"
