#!/bin/bash
# Runs GPU steps in order on the gpurun box; each step has its own time limit.  A step that ends
# with a signal/timeout/abort (rc >= 124) stops the script (no further GPU work in this call);
# ordinary failures (rc 1-2, e.g. a failing test) let later steps run.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/steps.log; exit $rc; fi
done
exit 0
