#!/bin/bash
# Runs a sequence of GPU steps on the box; stops at the first step that faults, aborts,
# segfaults or times out (exit codes other than 0/1).  usage: tools/gpu_run.sh "<cmd1>" "<cmd2>" ...
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a gpurun_out/steps.log
  bash -c "$cmd" > gpurun_out/step$i.log 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  tail -25 gpurun_out/step$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $i exited with $rc"; exit $rc
  fi
done
