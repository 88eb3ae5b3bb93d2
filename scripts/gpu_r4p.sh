#!/usr/bin/env bash
# ResNet-18 B=256: halo weight-gradient workgroup target A/B (split-m count -> slab reduce size)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for v in "" "halo_wg=128" "halo_wg=512" "halo_wg=192" ""; do
  DISTRIFLOW_DIAG=$v timeout -k 10 120 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 60 --warmup 10 --async-steps 0 > gpurun_out/b_rn_hw.json 2> gpurun_out/b_rn_hw.err || { tail -n 20 gpurun_out/b_rn_hw.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_rn_hw.json'));print('[$v]', d['value'], d['ms_per_step'])" | tee -a gpurun_out/rn_halo_wg_ab.txt
done
