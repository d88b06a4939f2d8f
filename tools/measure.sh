#!/bin/bash
# Round measurement on a 1-GPU MI355X box (run through gpurun from the repo root):
#   tools/measure.sh <tag> [config] [skip-tests]
# -> gpurun_out/pytest_gpu.log, gpurun_out/bench_<cfg>.json (the default bench line: groups and
#    cpu_baseline included), gpurun_out/prof/<cfg>_kernel_stats.csv (+ kernel trace),
#    gpurun_out/prof/pmc_{fetch,write}_counter_collection.csv, gpurun_out/pmc_<cfg>.json
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:?tag}
cfg=${2:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O/prof"
if [ "${3:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -v --durations=25 --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -1 "$O/pytest_gpu.log"
fi
timeout -k 10 400 python "$R/bench.py" --config "$cfg" > "$O/bench_$cfg.json" 2> "$O/bench_$cfg.err" || { tail -20 "$O/bench_$cfg.err"; exit 1; }
cat "$O/bench_$cfg.json"
cd /tmp && export TMPDIR=/tmp
P=(python3 "$R/bench.py" --config "$cfg" --no-cpu --groups '')
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o "$cfg" -- "${P[@]}" > "$O/prof_$cfg.json" 2> "$O/prof_$cfg.err" || { tail -20 "$O/prof_$cfg.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/prof" -o pmc_fetch -- "${P[@]}" > "$O/pmc_fetch.json" 2> "$O/pmc_fetch.err" || { tail -20 "$O/pmc_fetch.err"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/prof" -o pmc_write -- "${P[@]}" > "$O/pmc_write.json" 2> "$O/pmc_write.err" || { tail -20 "$O/pmc_write.err"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$O/prof" "$cfg" > "$O/pmc_$cfg.json"
echo "measure $tag $cfg done"
