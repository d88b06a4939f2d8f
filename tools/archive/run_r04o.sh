#!/bin/bash
# round 4 final-chain measurement: rocprofv3 kernel stats + FETCH/WRITE_SIZE passes of the C3
# line (tools/measure.sh), the chain's SQ counters (tools/chain_pmc.sh), and rocprofv3 kernel
# stats of the driver's exact bench command (tools/prof_driver_cmd.sh)
./tools/gpu_steps.sh \
 "1000 ./tools/measure.sh r04pk c3 skip-tests" \
 "300 ./tools/chain_pmc.sh fin2" \
 "1000 ./tools/prof_driver_cmd.sh"
