#!/usr/bin/env bash
# round-3 GPU session J: the reference CNN's dense head as one split-K launch (csrc/khead.hip)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_khead_gpu.py \
  tests/test_kcnn_fused_gpu.py tests/test_dropout_fold_gpu.py > gpurun_out/t_j.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_j.log | head -n 30; tail -n 40 gpurun_out/t_j.log; exit 1; }
tail -n 2 gpurun_out/t_j.log
timeout -k 10 300 python bench.py --model keras_cnn --batch-per-gpu 1024 --steps 200 --warmup 20 --async-steps 0 > gpurun_out/b_kc.log 2>&1 || { tail -n 30 gpurun_out/b_kc.log; exit 1; }
tail -n 1 gpurun_out/b_kc.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_kc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kc -o k --output-format csv -- python3 $R/bench.py --model keras_cnn --batch-per-gpu 1024 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_kc.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_kc.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_kc -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi > gpurun_out/prof_kc.txt
head -n 40 gpurun_out/prof_kc.txt
