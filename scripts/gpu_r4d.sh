#!/usr/bin/env bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
T="tests/test_fused_dp_gpu.py::test_fused_exchange_multistep_graph_matches_single_steps[2]"
for i in 1 2 3; do
timeout -k 10 200 python -u -m pytest "$T" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4d_$i.log 2>&1
echo "run $i rc=$?"; grep -E "passed|failed" gpurun_out/t_r4d_$i.log | tail -1
done
