#!/usr/bin/env bash
# round-3 session R: whole GPU suite with the halo kernels, headline bench, ResNet step breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_full.log 2>&1 || { grep -E "FAILED|ERROR|Error|assert" gpurun_out/t_full.log | head -n 30; tail -n 30 gpurun_out/t_full.log; exit 1; }
tail -n 1 gpurun_out/t_full.log
timeout -k 10 200 python bench.py > gpurun_out/b_lenet.log 2>&1 || { tail -n 20 gpurun_out/b_lenet.log; exit 1; }
tail -n 1 gpurun_out/b_lenet.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_rn -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi > gpurun_out/prof_rn.txt
cat gpurun_out/prof_rn.txt
