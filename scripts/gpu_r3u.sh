#!/usr/bin/env bash
# round-3 session U: reference-CNN dense head phase stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 120 python scripts/kheadstamps.py > gpurun_out/khs.txt 2>&1 || { tail -n 20 gpurun_out/khs.txt; exit 1; }
cat gpurun_out/khs.txt
for d in "" "conv_halo_ks=2" "conv_halo_splitk=0"; do
  DISTRIFLOW_DIAG=$d timeout -k 10 120 python scripts/convbench.py l4 > gpurun_out/cb_ks.txt 2>&1 || { tail -n 20 gpurun_out/cb_ks.txt; exit 1; }
  echo "diag=[$d] $(grep l4 gpurun_out/cb_ks.txt)"
done
for i in 1 2; do
for d in "" "conv_halo_ks=2" "conv_halo_splitk=0"; do
  DISTRIFLOW_DIAG=$d timeout -k 10 120 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 200 --warmup 10 --async-steps 0 > gpurun_out/b_ks.log 2>&1 || { tail -n 20 gpurun_out/b_ks.log; exit 1; }
  echo "diag=[$d] $(python3 -c "import json; d=json.loads(open('gpurun_out/b_ks.log').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
done
