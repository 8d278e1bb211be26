#!/bin/bash
# Run GPU steps in order; stop at the first step that fails (a fault, abort, time limit or error).
# usage: tools/gpurun/steps.sh "<limit_s> <name> <cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  limit=${spec%% *}; rest=${spec#* }; name=${rest%% *}; cmd=${rest#* }
  echo "== $name (limit ${limit}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
