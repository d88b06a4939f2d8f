#!/bin/bash
# C4's per-rank line on one MI355X at 64 and 128 slices, with the world-1 exchange at gain 1 (RCCL,
# stream plumbing + delta / apply kernels) and without
O=gpurun_out/c4_slices; mkdir -p $O
for k in 64 128; do
  for x in on off; do
    timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 --slices $k --ar-allreduce $x --xchg-gain 1 > $O/k${k}_$x.json 2> $O/k${k}_$x.err || { tail -20 $O/k${k}_$x.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/k${k}_$x.json')); print('$k', '$x', round(d['value']/1e6,3), round(d['ms_per_step'],2), d['stream_ms_per_step'], (d.get('ar_allreduce') or {}).get('ms_per_call_event_timed'))"
  done
done
