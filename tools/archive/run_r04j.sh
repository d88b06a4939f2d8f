#!/bin/bash
# AR chain unfenced: chain A/B, chain SQ counters, GPU suite, smoke, the driver's bench command
./tools/gpu_steps.sh \
 "300 ./tools/chain_ab.sh 2 b128 fa > gpurun_out/r04_chain_ab_fa.log 2>&1; tail -4 gpurun_out/r04_chain_ab_fa.log" \
 "300 ./tools/chain_pmc.sh fa" \
 "900 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_gputest_fa.txt 2>&1; tail -3 gpurun_out/r04_gputest_fa.txt" \
 "300 python3 -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_fa.json"
