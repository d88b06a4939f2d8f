#!/bin/bash
# Round 6's GPU jobs, one parameterised script (tools/gpu_steps.sh runs each step under its own
# time limit and stops after a fault or a timeout).   gpurun -- ./tools/r06.sh <job>
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
PYT="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
case "$1" in
  sched_kuhn)   # the group schedule test + C5 to 400M+ hands (item 6)
    ./tools/gpu_steps.sh \
      "400 $PYT tests/test_gpu_group.py tests/test_gpu_exchange.py -m gpu > $O/pytest_group.log" \
      "300 python3 -u tools/exploit_curve.py --config c5 --quirks 504 --set slices=16 --set slice_lag=2 --steps 420 --every 20 > $O/kuhn_tb_slices16.jsonl" \
      "300 python3 -u tools/exploit_curve.py --config c5 --set slices=16 --set slice_lag=2 --steps 420 --every 42 > $O/kuhn_ref_slices16.jsonl"
    ;;
  chain8)       # the 8-wave sample-split chain against k_chain3 (tools/bench_chain.hip)
    B=tools/bin/bench_chain_${2:-r06c8}_br
    ./tools/gpu_steps.sh \
      "60 for r in 1 0; do $B 200 \$r compare; CHAIN8=1 $B 200 \$r compare; CHAIN8=1 $B 2000 \$r compare; done > $O/chain8_compare.log" \
      "120 for r in 1 0; do for b in 1 2; do $B 2000 \$r time \$b; CHAIN8=1 $B 2000 \$r time \$b; done; done > $O/chain8_time.log"
    ;;
  kuhn_lr)      # C5 textbook MSE: lower learning rates against the 0.06-0.09 SGD-noise floor
    C5="python3 -u tools/exploit_curve.py --config c5 --quirks 504 --set slices=16 --set slice_lag=2 --steps 420 --every 20"
    ./tools/gpu_steps.sh \
      "300 $C5 --set lr_ar=0.02 > $O/kuhn_tb_lrar02.jsonl" \
      "300 $C5 --set lr_ar=0.02 --set lr_br=0.01 > $O/kuhn_tb_lrar02_lrbr01.jsonl" \
      "300 $C5 --set lr_ar=0.005 > $O/kuhn_tb_lrar005.jsonl"
    ;;
  kuhn_eps)     # C5 textbook MSE with the reference's decaying epsilon (no NFSP_EXT_EPS_CONST):
                # a constant 0.06 puts 6 % uniform-random actions into M_SL (one-hot argmax)
    C5="python3 -u tools/exploit_curve.py --config c5 --set slices=16 --set slice_lag=2 --steps 420 --every 20"
    ./tools/gpu_steps.sh \
      "300 $C5 --quirks 440 > $O/kuhn_tb_epsdecay.jsonl" \
      "300 $C5 --quirks 440 --set lr_ar=0.02 > $O/kuhn_tb_epsdecay_lrar02.jsonl"
    ;;
  stamps)
    B=tools/bin/bench_chain_${2:-r06st}_br
    ./tools/gpu_steps.sh "120 for r in 1 0; do $B 2000 \$r time; CHAIN8=1 $B 2000 \$r time; done > $O/chain8_stamps.log"
    ;;
  c3_seeds)     # C3's learning curve at 16 / 32 / 128 slices over 24 seeds
    for off in 0 8 16; do
      ./tools/gpu_steps.sh "600 python3 -u tests/studies/exploit_slices.py --steps 32 --every 8 --variants 16:2 128:2 32:2 --seed-offset $off > $O/c3_slices_seeds$off.json" || exit 1
    done
    ;;
  persist)      # k_br_persist's hand-off protocol and geometry, trivial work.
                # A host watchdog prints the kernel's progress counters and exits after 10 s.
    P=tools/bin/persist_probe
    ./tools/gpu_steps.sh \
      "20 $P 1 3 150 1048576 0 > $O/persist_big_lds.log" \
      "20 $P 2 3 150 1048576 0 > $O/persist_r2.log" \
      "20 $P 16 4 150 1048576 0 > $O/persist_r16.log" \
      "20 $P 2 3 150 2000 1 > $O/persist_r2_slow_bails.log" \
      "20 $P 2 3 150 1048576 16 > $O/persist_r2_devmem.log" \
      "20 $P 2 3 150 1048576 8 > $O/persist_r2_printf.log"
    ;;
  persist2)     # the first probes' exact host / atomics configuration, one factor at a time
    P=tools/bin/persist_probe
    ./tools/gpu_steps.sh \
      "20 $P 1 3 150 1048576 48 16384 > $O/persist2_sync_devmem.log" \
      "20 $P 1 3 150 1048576 112 16384 > $O/persist2_sync_devmem_agent.log" \
      "20 $P 1 3 150 1048576 120 16384 > $O/persist2_sync_devmem_agent_printf.log" \
      "20 $P 1 3 150 2000 120 > $O/persist2_v1.log"
    ;;
  final)        # the committed tree: the GPU suite, smoke(), the driver's bench command
    ./tools/gpu_steps.sh \
      "900 python3 -u -m pytest tests -m gpu -v --durations=15 --timeout 400 --timeout-method thread > $O/gputest_final.log" \
      "300 python3 -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > $O/smoke_final.log" \
      "600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_final.json"
    ;;
  prof)         # rocprofv3 --kernel-trace --stats of the driver's command, then the PMC passes
    R=$(pwd); D=$R/$O/prof; mkdir -p $D
    ( cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o drv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err &&
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D -o pmc_fetch -- python3 $R/bench.py --config c3 --no-cpu --groups '' > $D/pmc_fetch.json 2> $D/pmc_fetch.err &&
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D -o pmc_write -- python3 $R/bench.py --config c3 --no-cpu --groups '' > $D/pmc_write.json 2> $D/pmc_write.err ) || { tail -20 $D/*.err; exit 1; }
    python3 tools/pmc_summary.py $D c3 > $O/pmc_c3_r06.json
    find $D -name "*stats*"
    ;;
  all)          # the final validation, the profiles, then the persist probe variants (last: a
                # variant may hang, and a timeout ends the call)
    ./tools/r06.sh final && ./tools/r06.sh prof && ./tools/r06.sh persist2
    ;;
  c4w1)         # C4's per-rank line with the RCCL exchange at world 1, on the final bench.py
    ./tools/gpu_steps.sh \
      "300 python3 -u bench.py --config c4 --ar-allreduce on --no-cpu --groups '' --steps 10 --warmup 3 > $O/c4_rank_xchg_world1.json"
    ;;
  more_seeds)   # C4's emulation over 16 more seeds; C3 to 134M hands over 8 seeds
    ./tools/gpu_steps.sh \
      "600 python3 -u tests/studies/c4_gate_seeds.py --seeds 8 24 > $O/c4_gate_seeds8_23.json" \
      "600 python3 -u tests/studies/exploit_slices.py --steps 128 --every 16 --variants 16:2 > $O/c3_long_128steps.json"
    ;;
  chain_ab)     # A/B of two chain microbenchmark builds: tools/r06.sh chain_ab <tagA> <tagB>
    A=tools/bin/bench_chain_$2_br; B=tools/bin/bench_chain_$3_br
    ./tools/gpu_steps.sh \
      "60 for r in 1 0; do $A 200 \$r compare; $B 200 \$r compare; done > $O/chain_ab_$2_$3_compare.log" \
      "200 for i in 1 2 3; do for r in 1 0; do $A 2000 \$r time; $B 2000 \$r time; done; done > $O/chain_ab_$2_$3_time.log"
    ;;
  brp)          # k_br_persist re-landed (profiles/r06/persist_rootcause): the group suite, then
                # c4_emul_r8 with the rounds and with the persistent kernel in one bench process
    ./tools/gpu_steps.sh \
      "900 $PYT tests/test_gpu_group.py > $O/brp_group_tests.log" \
      "900 python3 -u bench.py --no-cpu --groups c4_emul_r8,c4_emul_r8_persist --steps 5 --warmup 2 > $O/brp_bench_groups.json"
    ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
