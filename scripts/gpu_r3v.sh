#!/usr/bin/env bash
# round-3 session V: halo conv split 2 by default; conv numerics; ResNet bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo or splitk or conv" \
  > gpurun_out/t_v.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_v.log | head -n 30; tail -n 30 gpurun_out/t_v.log; exit 1; }
tail -n 1 gpurun_out/t_v.log
timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_v.txt 2>&1 || { tail -n 20 gpurun_out/cb_v.txt; exit 1; }
cat gpurun_out/cb_v.txt
for i in 1 2; do
timeout -k 10 120 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 200 --warmup 10 --async-steps 0 > gpurun_out/b_rn_v.log 2>&1 || { tail -n 20 gpurun_out/b_rn_v.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_rn_v.log').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])"
done
DISTRIFLOW_DIAG=conv_halo_pitch16=0 timeout -k 10 200 python scripts/convbench.py l2 > gpurun_out/cb_v2.txt 2>&1 || { tail -n 20 gpurun_out/cb_v2.txt; exit 1; }
echo "pitch16=0: $(grep l2 gpurun_out/cb_v2.txt)"
for i in 1 2; do
DISTRIFLOW_DIAG=conv_halo_pitch16=0 timeout -k 10 120 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 200 --warmup 10 --async-steps 0 > gpurun_out/b_rn_v.log 2>&1 || { tail -n 20 gpurun_out/b_rn_v.log; exit 1; }
echo "pitch16=0: $(python3 -c "import json; d=json.loads(open('gpurun_out/b_rn_v.log').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
