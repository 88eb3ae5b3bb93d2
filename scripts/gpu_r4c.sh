#!/usr/bin/env bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
F="amdgpu.ids\|Gloo\|socket.cpp"
timeout -k 10 200 python -u scripts/dbg_selftest_state.py 2>&1 | grep -v "$F" && \
timeout -k 10 200 python -u scripts/ll_bench.py 2 2>&1 | grep -v "$F" | tee gpurun_out/ll_bench_2r.txt && \
timeout -k 10 200 python -u scripts/lenetstamps.py 4096 step 2>&1 | grep -v "$F" | tee gpurun_out/lenetstamps_sync.txt && \
timeout -k 10 200 python -u scripts/lenetstamps.py 4096 async 2>&1 | grep -v "$F" | tee gpurun_out/lenetstamps_async.txt
