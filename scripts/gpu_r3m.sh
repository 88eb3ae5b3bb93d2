#!/usr/bin/env bash
# round-3 session M: halo-tiled 3x3 forward / data gradient (csrc/conv3_halo.hip) + wgrad workgroup sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo or conv" \
  > gpurun_out/t_m.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_m.log | head -n 30; tail -n 30 gpurun_out/t_m.log; exit 1; }
tail -n 1 gpurun_out/t_m.log
timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_m.txt 2>&1 || { tail -n 20 gpurun_out/cb_m.txt; exit 1; }
cat gpurun_out/cb_m.txt
for wg in 256 1024; do
  DISTRIFLOW_DIAG=halo_wg=$wg timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_wg$wg.txt 2>&1 || { tail -n 20 gpurun_out/cb_wg$wg.txt; exit 1; }
  echo "halo_wg=$wg"; grep -o "wgrad.*" gpurun_out/cb_wg$wg.txt
done
timeout -k 10 300 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 50 --warmup 10 --async-steps 0 > gpurun_out/b_rn_m.log 2>&1 || { tail -n 20 gpurun_out/b_rn_m.log; exit 1; }
tail -n 1 gpurun_out/b_rn_m.log
