#!/usr/bin/env bash
# khead: tests, bench, stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_khead_gpu.py > gpurun_out/t_q.log 2>&1 || { tail -n 30 gpurun_out/t_q.log; exit 1; }
tail -n 1 gpurun_out/t_q.log
timeout -k 10 120 python bench.py --model keras_cnn --batch-per-gpu 1024 --steps 200 --warmup 20 --async-steps 0 > gpurun_out/b_q.log 2>&1 || { tail -n 20 gpurun_out/b_q.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_q.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
timeout -k 10 120 python scripts/kheadstamps.py > gpurun_out/khs_q.txt 2>&1 || { tail -n 20 gpurun_out/khs_q.txt; exit 1; }
sed -n 3,12p gpurun_out/khs_q.txt
