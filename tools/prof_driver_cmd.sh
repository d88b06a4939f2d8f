#!/bin/bash
# rocprofv3 kernel statistics of the driver's exact bench command (the roofline kernel's
# average launch duration, compared with the line's live HIP-event figure)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_driver
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o drv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
ls $O
