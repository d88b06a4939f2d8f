#!/usr/bin/env python3
"""Engine step time with RCCL initialised in the same process (diagnostic): a
world-size-1 NCCL (RCCL) process group is created first, as bench.py does for N > 1, then a
C3 engine; 2 warmup + 5 timed steps, each followed by the AR all-reduce.
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29541 tools/rccl_streams_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))   # world 1: RCCL's streams exist
world = dist.get_world_size()
print("world", world, "queues", os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
import __graft_entry__
pkg = __graft_entry__.load_package()
eng = pkg.engine.SelfPlayEngine(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000, seed=1234, init_seed=0)
avg = pkg.shards.AvgPolicyAllReduce([eng.weights_tensor(a, pkg.engine.NET_AR) for a in (0, 1)], dist, sync=torch.cuda.synchronize) if dist else None
def step():
    eng.step()
    if avg: avg()
for _ in range(2): step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5): step()
torch.cuda.synchronize()
print(json.dumps({"ms_per_step": (time.perf_counter() - t0) / 5 * 1e3}), flush=True)
if dist: dist.destroy_process_group()
