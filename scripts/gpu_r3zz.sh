#!/usr/bin/env bash
# round-3 final profiles: ResNet-18 step breakdown on the final defaults, LeNet-5 step kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/prof_rn $R/gpurun_out/prof_ln
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ln -o k --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --async-steps 0 > $R/gpurun_out/prof_ln.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_ln.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_rn -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi > gpurun_out/prof_rn.txt
cat gpurun_out/prof_rn.txt
f=$(find gpurun_out/prof_ln -name '*kernel_stats.csv' | head -n 1)
head -n 8 "$f"
