#!/bin/bash
# round 4, packed f32 (BR: W update; AR: W update + softmax pairs): microbenchmark vs the
# scalar chain, the CU-sharing group probe, the GPU suite, bench.py with the driver's command
./tools/gpu_steps.sh \
 "120 ./tools/ar_var.sh 3 base fin2 -- base fin2" \
 "200 python3 -u tools/group_share_probe.py 200 4" \
 "120 python3 -u tools/group_share_probe.py 80 2" \
 "200 NFSP_LIB=tools/bin/libnfsp_brl2.so python3 -u tools/group_share_probe.py 200 3" \
 "700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_pk2.json"
