#!/usr/bin/env bash
# reduce-launch bandwidth probe: stamps with dense loads / conv loads skipped
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for p in 0 1 2; do
  echo "=== lenet_red_probe=$p"
  DISTRIFLOW_DIAG=lenet_red_probe=$p timeout -k 10 200 python scripts/lenetstamps.py 4096 step > gpurun_out/stamps_p$p.log 2>&1 || { tail -n 30 gpurun_out/stamps_p$p.log; exit 1; }
  grep -A 10 "dense  jobs" gpurun_out/stamps_p$p.log
done
