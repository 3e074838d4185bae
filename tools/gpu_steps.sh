#!/bin/bash
# Run GPU steps in sequence on the gpurun box; each step has its own time limit and log under gpurun_out/.
# A step that fails normally (tests failing: rc 1/2) does not stop the sequence; a fault, abort, segfault, time
# limit or kill (rc 124 / 134 / 137 / 139 / >128) ends the script there.
#   usage: tools/gpu_steps.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/steps.log
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc $rc: stopping"; exit $rc; fi
done
