#!/usr/bin/env bash
# round-3 GPU session A: fused multi-rank LeNet-5 step (in-kernel LL exchange), fused async PS step,
# generic-layer kernels, 1-GPU bench, 2-rank rehearsal bench and per-rank kernel traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
run_tests() {  # name, files...
  local name=$1; shift
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/t_$name.log 2>&1
  local rc=$?
  tail -n 4 gpurun_out/t_$name.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/t_$name.log | head -n 30; exit 1; fi
}
run_tests kern tests/test_lenet_fused_gpu.py tests/test_general_kernels_gpu.py tests/test_engine_gpu.py
run_tests fused tests/test_fused_dp_gpu.py tests/test_p2p_gpu.py
run_tests async tests/test_async_ps_gpu.py
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/b1.log 2>&1 || { cat gpurun_out/b1.log; exit 1; }
cat gpurun_out/b1.log
DISTRIFLOW_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/b2.log 2>&1 || { cat gpurun_out/b2.log; exit 1; }
cat gpurun_out/b2.log
scripts/prof_ranks.sh 2 --steps 30 --warmup 5 --async-steps 0 > gpurun_out/prof2.log 2>&1 || { tail -n 30 gpurun_out/prof2.log; exit 1; }
cat gpurun_out/prof2.log
