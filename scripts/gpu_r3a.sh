#!/usr/bin/env bash
# round-3 GPU session A: fused multi-rank LeNet-5 step (in-kernel LL exchange) tests, 1-GPU bench,
# 2-rank rehearsal bench and per-rank kernel traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fused_dp_gpu.py tests/test_p2p_gpu.py tests/test_lenet_fused_gpu.py tests/test_engine_gpu.py tests/test_general_kernels_gpu.py > gpurun_out/t_fused.log 2>&1 || { tail -n 40 gpurun_out/t_fused.log; exit 1; }
tail -n 15 gpurun_out/t_fused.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/b1.log 2>&1 || { cat gpurun_out/b1.log; exit 1; }
cat gpurun_out/b1.log
DISTRIFLOW_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --steps 20 --warmup 5 --async-steps 0 > gpurun_out/b2.log 2>&1 || { cat gpurun_out/b2.log; exit 1; }
cat gpurun_out/b2.log
scripts/prof_ranks.sh 2 --steps 30 --warmup 5 --async-steps 0 > gpurun_out/prof2.log 2>&1 || { tail -n 30 gpurun_out/prof2.log; exit 1; }
cat gpurun_out/prof2.log
