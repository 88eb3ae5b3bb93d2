#!/usr/bin/env bash
# 128-channel halo conv with a kernel row per step and the compact halo (conv_halo_row128): numerics with
# it on, per-conv timing A/B, ResNet-18 bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
DISTRIFLOW_DIAG=conv_halo_row128=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4y.log 2>&1 || { tail -n 30 gpurun_out/t_r4y.log; exit 1; }
tail -n 1 gpurun_out/t_r4y.log
for v in conv_halo_row128=0 conv_halo_row128=1; do
  echo "== $v"
  DISTRIFLOW_DIAG=$v timeout -k 10 200 python3 scripts/convbench.py l2 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in conv_halo_row128=0 conv_halo_row128=1 conv_halo_row128=0 conv_halo_row128=1; do
  DISTRIFLOW_DIAG=$v timeout -k 10 200 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 60 --warmup 10 --async-steps 0 > gpurun_out/b_rn_r128.json 2> gpurun_out/b_rn_r128.err || { tail -n 20 gpurun_out/b_rn_r128.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/b_rn_r128.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
