#!/usr/bin/env bash
# ResNet-18 BN statistics sizing A/B (rows per thread -> workgroups per statistics launch)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for v in 16 4 8 32; do
  DISTRIFLOW_DIAG=bn_rpt=$v timeout -k 10 200 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 60 --warmup 10 --async-steps 0 > gpurun_out/b_rn_rpt$v.json 2> gpurun_out/b_rn_rpt$v.err || { tail -n 20 gpurun_out/b_rn_rpt$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_rn_rpt$v.json'));print('bn_rpt=$v', d['value'], d['ms_per_step'])"
done
