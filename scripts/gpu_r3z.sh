#!/usr/bin/env bash
# round-3 session Z: ResNet-18 with in-order weight gradients (new default) - engine tests + A/B of the rest
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py > gpurun_out/t_z.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_z.log | head -n 20; tail -n 20 gpurun_out/t_z.log; exit 1; }
tail -n 1 gpurun_out/t_z.log
: > gpurun_out/ab_z.txt
for i in 1 2; do
  for d in "" "proj_overlap=0" "halo_groups=1" "wgrad_overlap=1"; do
    DISTRIFLOW_DIAG=$d timeout -k 10 120 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 200 --warmup 10 --async-steps 0 > gpurun_out/b_z.log 2>&1 || { tail -n 20 gpurun_out/b_z.log; exit 1; }
    echo "diag=[$d] $(python3 -c "import json; d=json.loads(open('gpurun_out/b_z.log').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")" | tee -a gpurun_out/ab_z.txt
  done
done
