#!/bin/bash
# Run GPU steps in sequence; continue past ordinary test failures (rc 1) but stop after a
# fault, abort, segfault or timeout (any other non-zero rc) -- nothing more touches the GPU then.
# usage: tools/gpu_steps.sh "<seconds> <cmd...>" "<seconds> <cmd...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%% *}
  cmd=${spec#* }
  echo "=== [$secs s] $cmd"
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: rc=$rc"
    exit $rc
  fi
done
