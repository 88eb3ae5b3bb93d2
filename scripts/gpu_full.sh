#!/usr/bin/env bash
# the whole GPU test suite (round-end rehearsal), one process, per-test time limits
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_full.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/t_full.log | tail -n 30
exit $rc
