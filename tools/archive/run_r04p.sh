#!/bin/bash
# round 4, packed chains: the other configs' lines (C2, C5, C5 textbook) and C4's per-rank
# line on one MI355X with the world-1 RCCL exchange (gain 2, as deployed) and without
O=gpurun_out/c4_pk; mkdir -p $O
./tools/gpu_steps.sh \
 "900 ./tools/run_configs.sh r04pk c2 c5 c5_tb" \
 "300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 --ar-allreduce on > $O/c4_on.json" \
 "300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 --ar-allreduce off > $O/c4_off.json"
for x in on off; do python3 -c "import json; d=json.load(open('$O/c4_$x.json')); print('c4 $x', round(d['value']/1e6,3), round(d['ms_per_step'],2), d['stream_ms_per_step'], (d.get('ar_allreduce') or {}).get('ms_per_call_event_timed'))"; done
