#!/usr/bin/env bash
# FedSGD barrier imbalance diagnosis: LeNet CPU-reference shapes + fedsgd k = 8 / 6 / 5 (no -x)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_dp_gpu.py -k "fedsgd or union" -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4f.log 2>&1
grep -E "passed|failed|Error|rel" gpurun_out/t_r4f.log | tail -n 20
