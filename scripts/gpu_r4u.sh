#!/usr/bin/env bash
# Halo conv with a kernel row per step (conv_halo_row): numerics, per-conv timing A/B, ResNet-18 bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo or splitk" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4u.log 2>&1 || { tail -n 30 gpurun_out/t_r4u.log; exit 1; }
tail -n 1 gpurun_out/t_r4u.log
for v in conv_halo_row=0 conv_halo_row=1; do
  echo "== $v"
  DISTRIFLOW_DIAG=$v timeout -k 10 200 python3 scripts/convbench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/convbench_$v.txt || exit 1
done
for v in conv_halo_row=0 conv_halo_row=1 conv_halo_row=0 conv_halo_row=1; do
  DISTRIFLOW_DIAG=$v timeout -k 10 200 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 60 --warmup 10 --async-steps 0 > gpurun_out/b_rn_row.json 2> gpurun_out/b_rn_row.err || { tail -n 20 gpurun_out/b_rn_row.err; exit 1; }
  echo "$v $(cut -c1-200 gpurun_out/b_rn_row.json)"
done
