#!/usr/bin/env bash
# round-3 session X: steps-per-graph chosen so the warm-up replays the timed graph (driver K=20 / W=5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/b_x.log 2>&1 || { tail -n 20 gpurun_out/b_x.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_x.log').read().strip().splitlines()[-1]); print('K20', round(d['value']), d['ms_per_step'], d['config']['steps_per_graph'], d['async']['speedup_vs_sync'])"
done
timeout -k 10 200 python bench.py > gpurun_out/b_x.log 2>&1 || { tail -n 20 gpurun_out/b_x.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_x.log').read().strip().splitlines()[-1]); print('K200', round(d['value']), d['ms_per_step'], d['config']['steps_per_graph'], d['async']['speedup_vs_sync'])"
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_bench_contract.py > gpurun_out/t_x.log 2>&1 || { tail -n 30 gpurun_out/t_x.log; exit 1; }
tail -n 1 gpurun_out/t_x.log
