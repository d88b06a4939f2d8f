#!/bin/bash
# round 4 measurement of the final tree: the driver's bench command, the rocprof kernel stats
# and PMC passes of the C3 line, and C4's per-rank line with and without the exchange at world 1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O/prof"
./tools/gpu_steps.sh \
 "400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench_driver_cmd.json" \
 "300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 > gpurun_out/r04_c4_rank_noxchg.json" \
 "300 python3 -u bench.py --config c4 --no-cpu --groups '' --steps 10 --warmup 3 --ar-allreduce on --xchg-gain 1 > gpurun_out/r04_c4_rank_xchg_world1.json" || exit 1
cd /tmp && export TMPDIR=/tmp
P=(python3 "$R/bench.py" --config c3 --no-cpu --groups '')
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o c3 -- "${P[@]}" > "$O/prof_c3.json" 2> "$O/prof_c3.err" || { tail -20 "$O/prof_c3.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/prof" -o pmc_fetch -- "${P[@]}" > "$O/pmc_fetch.json" 2> "$O/pmc_fetch.err" || { tail -20 "$O/pmc_fetch.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/prof" -o pmc_write -- "${P[@]}" > "$O/pmc_write.json" 2> "$O/pmc_write.err" || { tail -20 "$O/pmc_write.err"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$O/prof" c3 > "$O/pmc_c3.json"
ls "$O/prof" | head
echo "r04c done"
