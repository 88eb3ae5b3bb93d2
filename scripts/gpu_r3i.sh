#!/usr/bin/env bash
# round-3 GPU session I: ResNet-18 with BatchNorm statistics inside the conv launches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "bn_ or resnet" \
  tests/test_callbacks_gpu.py > gpurun_out/t_i.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_i.log | head -n 30; tail -n 40 gpurun_out/t_i.log; exit 1; }
tail -n 2 gpurun_out/t_i.log
timeout -k 10 300 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 30 --warmup 5 --async-steps 0 > gpurun_out/b_rn.log 2>&1 || { tail -n 30 gpurun_out/b_rn.log; exit 1; }
tail -n 1 gpurun_out/b_rn.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 10 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_rn -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi > gpurun_out/prof_rn.txt
head -n 40 gpurun_out/prof_rn.txt
