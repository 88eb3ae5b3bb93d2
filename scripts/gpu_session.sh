#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time limit, and the session
# stops at the first step that crashes / aborts / times out (exit codes other than 0 and 1), so a
# GPU fault never gets a second kernel launched after it.
#   usage: scripts/gpu_session.sh "<timeout_s> <name> <command...>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  t=$(echo "$spec" | awk '{print $1}')
  name=$(echo "$spec" | awk '{print $2}')
  cmd=$(echo "$spec" | cut -d' ' -f3-)
  echo "=== [$name] ($t s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc ($(( $(date +%s) - start )) s)" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping session after rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
