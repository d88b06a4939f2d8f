#!/bin/bash
# C3 (no process group) and C4's per-rank line with the world-1 RCCL exchange (nccl process
# group + libnfsp's communicator) under GPU_MAX_HW_QUEUES 4 / 8 / 16
mkdir -p gpurun_out/hwq
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --no-cpu --groups '' --steps 5 --warmup 2 > gpurun_out/hwq/c3_q$q.json || exit 1
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 5 --warmup 2 --ar-allreduce on --xchg-gain 1 > gpurun_out/hwq/c4x_q$q.json || exit 1
done
for f in gpurun_out/hwq/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e6,3), round(d['ms_per_step'],1), round(d['ms_per_step_event_timed'],1), {k: round(v,1) for k,v in d['stream_ms_per_step'].items()}, round(d['kernel_ms_per_step']['k_scan'],2))"; done
