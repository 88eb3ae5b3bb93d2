#!/usr/bin/env bash
# ResNet-18 B=256 in-order step breakdown (rocprofv3 kernel trace) + bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_rn -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi --order > gpurun_out/prof_rn.txt
head -n 40 gpurun_out/prof_rn.txt
timeout -k 10 300 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 100 --warmup 10 > gpurun_out/b_rn.json 2> gpurun_out/b_rn.err || { tail -n 20 gpurun_out/b_rn.err; exit 1; }
cat gpurun_out/b_rn.json
