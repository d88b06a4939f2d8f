#!/bin/bash
# round 4: the C4 gate (per-slice exchange), the saturated AR regime, and the long-horizon
# C4 curve (64 slices, gain 2, 24 steps = 201M hands, 8 seeds) -> profiles/r04_*
./tools/gpu_steps.sh \
 "300 python3 -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_learner_saturated.py" \
 "500 python3 -u -m pytest -x -v -s --timeout 480 --timeout-method thread tests/test_gpu_slices.py -k c4_emulated" \
 "600 python3 -u tests/studies/exploit_group.py --replicas 8 --lanes 8388608 --every 8388608 --hands 201326592 --seeds 8 --slices 64 --slice-lag 2 --xchg-every 1 --xchg-scale 0.25 > gpurun_out/r04_exploit_c4_slice_exchange.json"
