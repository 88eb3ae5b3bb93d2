#!/usr/bin/env bash
# A/B of the khead operand-hoisting variants (DISTRIFLOW_DIAG khead_hoist=0..3): bench + stamps each
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_khead_gpu.py > gpurun_out/t_ab.log 2>&1 || { tail -n 30 gpurun_out/t_ab.log; exit 1; }
tail -n 1 gpurun_out/t_ab.log
for h in 0 1 2 3; do
  DISTRIFLOW_DIAG=khead_hoist=$h timeout -k 10 120 python bench.py --model keras_cnn --batch-per-gpu 1024 --steps 200 --warmup 20 --async-steps 0 > gpurun_out/b_ab$h.log 2>&1 || { tail -n 20 gpurun_out/b_ab$h.log; exit 1; }
  echo "hoist=$h $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/b_ab$h.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  DISTRIFLOW_DIAG=khead_hoist=$h timeout -k 10 120 python scripts/kheadstamps.py > gpurun_out/khs$h.txt 2>&1 || { tail -n 20 gpurun_out/khs$h.txt; exit 1; }
  sed -n 3,12p gpurun_out/khs$h.txt
done
