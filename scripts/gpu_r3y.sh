#!/usr/bin/env bash
# round-3 session Y: ResNet-18 stream-overlap A/B with the halo kernels (alternating, 3 x 200 steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
: > gpurun_out/ab_ov.txt
for i in 1 2 3; do
  for d in "" "wgrad_overlap=0" "proj_overlap=0" "halo_groups=1"; do
    DISTRIFLOW_DIAG=$d timeout -k 10 120 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 200 --warmup 10 --async-steps 0 > gpurun_out/b_ov.log 2>&1 || { tail -n 20 gpurun_out/b_ov.log; exit 1; }
    echo "diag=[$d] $(python3 -c "import json; d=json.loads(open('gpurun_out/b_ov.log').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")" | tee -a gpurun_out/ab_ov.txt
  done
done
