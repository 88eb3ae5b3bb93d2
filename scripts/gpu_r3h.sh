#!/usr/bin/env bash
# round-3 GPU session H: LeNet correctness + bench + PMC (conflicts / waits)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_lenet_fused_gpu.py tests/test_fused_dp_gpu.py > gpurun_out/t_h.log 2>&1 \
  || { grep -E "FAILED|Error" gpurun_out/t_h.log | head -n 30; tail -n 30 gpurun_out/t_h.log; exit 1; }
tail -n 2 gpurun_out/t_h.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --async-steps 0 > gpurun_out/b1.log 2>&1 || { cat gpurun_out/b1.log; exit 1; }
cat gpurun_out/b1.log
bash scripts/pmc_lenet.sh > gpurun_out/pmc_lenet.log 2>&1 || { tail -n 20 gpurun_out/pmc_lenet.log; exit 1; }
cd "$R"
grep -A 1 "lenet_" gpurun_out/pmc_lenet_summary.txt
timeout -k 10 200 python scripts/lenetstamps.py 4096 > gpurun_out/stamps.log 2>&1 || { tail -n 30 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
