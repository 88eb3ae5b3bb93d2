#!/usr/bin/env bash
# A/B: the fused multi-rank multistep test with and without the real-kernel self-test
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
T="tests/test_fused_dp_gpu.py::test_fused_exchange_multistep_graph_matches_single_steps[2]"
DISTRIFLOW_DIAG=fused_selftest=0 timeout -k 10 300 python -u -m pytest "$T" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4b_off.log 2>&1
echo "selftest off rc=$?"; grep -E "PASSED|FAILED|Error" gpurun_out/t_r4b_off.log | head
timeout -k 10 300 python -u -m pytest "$T" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4b_on.log 2>&1
echo "selftest on rc=$?"; grep -E "PASSED|FAILED|Error" gpurun_out/t_r4b_on.log | head
