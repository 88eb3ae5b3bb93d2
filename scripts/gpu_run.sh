#!/usr/bin/env bash
# One parameterised GPU session (replaces the per-experiment gpu_r*.sh lease scripts).
#   scripts/gpu_run.sh <step> [<step> ...]    each step: "<timeout_s>|<name>|<command>"
# Every step runs under its own time limit with output in gpurun_out/<name>.log; the session stops at
# the first step that fails (any non-zero code), so nothing else touches the GPU after a fault or hang.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for spec in "$@"; do
  t=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "=== [$name] ($t s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc ($(( $(date +%s) - start )) s)"
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "session stopped after [$name] rc=$rc"; exit $rc; fi
done
