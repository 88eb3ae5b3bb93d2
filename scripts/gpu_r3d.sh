#!/usr/bin/env bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python scripts/lenetstamps.py 4096 step > gpurun_out/stamps.log 2>&1 || { tail -n 30 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
