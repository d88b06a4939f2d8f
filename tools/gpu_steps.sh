#!/bin/bash
# Run GPU steps one after another, each under its own time limit; stop at the first step that
# faulted, aborted or timed out (exit 124 / 134 / 137 / 139): nothing more touches the GPU then.
# Usage: tools/gpu_steps.sh "<seconds> <command>" ...   (logs: gpurun_out/step_<i>.log)
mkdir -p gpurun_out
i=0
for s in "$@"; do
  i=$((i + 1))
  t=${s%% *}; cmd=${s#* }
  echo "== step $i (limit $t s): $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > gpurun_out/step_$i.log 2>&1
  rc=$?
  tail -15 gpurun_out/step_$i.log
  echo "== step $i rc=$rc"
  case $rc in 124|134|137|139) echo "stopping: step $i ended with $rc"; exit $rc ;; esac
done
