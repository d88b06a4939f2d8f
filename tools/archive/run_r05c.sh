#!/bin/bash
# round 5: rocprofv3 kernel statistics of the driver's exact bench command, then the two PMC
# passes (separate runs, FETCH_SIZE / WRITE_SIZE) of the headline config for `traffic`
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_r05
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "== rocprofv3 --kernel-trace --stats of the driver's command"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o drv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
P=(python3 "$R/bench.py" --config c3 --no-cpu --groups '')
echo "== PMC FETCH_SIZE"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o pmc_fetch -- "${P[@]}" > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
echo "== PMC WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O -o pmc_write -- "${P[@]}" > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
python3 "$R/tools/pmc_summary.py" $O c3 > $R/gpurun_out/pmc_c3_r05.json
find $O -name "*stats*" | head; echo done
