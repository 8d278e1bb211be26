#!/bin/bash
# Run GPU steps in order; stop at the first step that faulted, aborted or timed out.
# usage: tools/gpu_steps.sh "<limit_s> <name> <cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  limit=${spec%% *}; rest=${spec#* }; name=${rest%% *}; cmd=${rest#* }
  echo "== $name (limit ${limit}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  case $rc in 124|134|137|139|-6|-11) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
done
