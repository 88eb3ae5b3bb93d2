#!/usr/bin/env bash
# round-3 session L: halo-tiled 3x3 weight gradient (csrc/wgrad_halo.hip): numerics, per-layer timing, ResNet-18
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" \
  > gpurun_out/t_l.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_l.log | head -n 30; tail -n 30 gpurun_out/t_l.log; exit 1; }
tail -n 1 gpurun_out/t_l.log
timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_halo.txt 2>&1 || { tail -n 20 gpurun_out/cb_halo.txt; exit 1; }
cat gpurun_out/cb_halo.txt
DISTRIFLOW_DIAG=wgrad_halo=0 timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_tr.txt 2>&1 || { tail -n 20 gpurun_out/cb_tr.txt; exit 1; }
cat gpurun_out/cb_tr.txt
timeout -k 10 300 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 50 --warmup 10 --async-steps 0 > gpurun_out/b_rn.log 2>&1 || { tail -n 20 gpurun_out/b_rn.log; exit 1; }
tail -n 1 gpurun_out/b_rn.log
