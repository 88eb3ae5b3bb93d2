#!/usr/bin/env bash
# round-3 session O: conv3_halo with a two-step weight register ring; wgrad groups A/B inside the model
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo" \
  > gpurun_out/t_o.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_o.log | head -n 30; tail -n 30 gpurun_out/t_o.log; exit 1; }
tail -n 1 gpurun_out/t_o.log
timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_o.txt 2>&1 || { tail -n 20 gpurun_out/cb_o.txt; exit 1; }
cat gpurun_out/cb_o.txt
for d in "" "halo_groups=1" "conv_halo_splitk=0"; do
  DISTRIFLOW_DIAG=$d timeout -k 10 300 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 100 --warmup 10 --async-steps 0 > gpurun_out/b_rn_o.log 2>&1 || { tail -n 20 gpurun_out/b_rn_o.log; exit 1; }
  echo "diag=$d $(python3 -c "import json; d=json.loads(open('gpurun_out/b_rn_o.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
