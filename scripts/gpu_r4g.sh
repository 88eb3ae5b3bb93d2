#!/usr/bin/env bash
# round-4 checkpoint: the whole GPU suite, smoke(), then the LeNet PMC passes (LDS conflicts, VALU / MFMA)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 420 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_r4g.log 2>&1; rc=$?
tail -n 15 gpurun_out/t_r4g.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4g.log 2>&1 || { tail -n 20 gpurun_out/smoke_r4g.log; exit 1; }
tail -n 1 gpurun_out/smoke_r4g.log
bash scripts/pmc_lenet.sh > gpurun_out/pmc_lenet.log 2>&1 || { tail -n 20 gpurun_out/pmc_lenet.log; exit 1; }
grep -A 1 "lenet_" gpurun_out/pmc_lenet_summary.txt
