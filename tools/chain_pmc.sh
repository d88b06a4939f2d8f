#!/bin/bash
# SQ counters of the SGD chain (microbenchmark, one chain = one workgroup of 4 waves), two
# passes of <= 8 SQ counters each (run through gpurun from the repo root):
#   tools/chain_pmc.sh <tag>   ->  gpurun_out/chain_pmc/<tag>_{br,ar}_p{1,2}/...
set -o pipefail
tag=${1:-base}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chain_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
for net in br ar; do
  relu=1; [ $net = ar ] && relu=0
  for p in 1 2; do
    C=P$p
    timeout -s KILL 60 rocprofv3 --pmc ${!C} --output-format csv -d $O/${tag}_${net}_p$p -o pmc -- $R/tools/bin/bench_chain_${tag}_$net 400 $relu time 1 > $O/${tag}_${net}_p$p.log 2>&1 || { tail -5 $O/${tag}_${net}_p$p.log; exit 1; }
  done
done
echo chain_pmc done
