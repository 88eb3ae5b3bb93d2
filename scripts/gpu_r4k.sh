#!/usr/bin/env bash
# ResNet-18 BN statistics workgroup cap A/B (bn_max_g) x rows per thread
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for v in "bn_max_g=255" "bn_max_g=512" "bn_max_g=1008" "bn_max_g=1008,bn_rpt=8" "bn_max_g=1008,bn_rpt=4" "bn_max_g=255"; do
  DISTRIFLOW_DIAG=$v timeout -k 10 120 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 60 --warmup 10 --async-steps 0 > gpurun_out/b_rn_ab.json 2> gpurun_out/b_rn_ab.err || { tail -n 20 gpurun_out/b_rn_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_rn_ab.json'));print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/rn_bn_grid_ab.txt
done
