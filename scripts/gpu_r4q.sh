#!/usr/bin/env bash
# reference CNN head change: head tests, bench, head stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "khead or keras or kcnn" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4q.log 2>&1 || { tail -n 30 gpurun_out/t_r4q.log; exit 1; }
tail -n 1 gpurun_out/t_r4q.log
for i in 1 2; do
timeout -k 10 200 python3 bench.py --model keras_cnn --batch-per-gpu 1024 --steps 100 --warmup 10 --async-steps 0 > gpurun_out/b_kc.json 2> gpurun_out/b_kc.err || { tail -n 20 gpurun_out/b_kc.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b_kc.json'));print('keras_cnn', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python3 scripts/kheadstamps.py > gpurun_out/kheadstamps.txt 2>&1 || { tail -n 20 gpurun_out/kheadstamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/kheadstamps.txt | head -n 13
