#!/usr/bin/env bash
# ResNet-18 B=256 on the final round-4 tree: bench (100 steps) and the per-kernel step breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 100 --warmup 10 > gpurun_out/b_rn_final.json 2> gpurun_out/b_rn_final.err || { tail -n 20 gpurun_out/b_rn_final.err; exit 1; }
cut -c1-300 gpurun_out/b_rn_final.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
f=$(ls $R/gpurun_out/prof_rn/*/*kernel_trace.csv $R/gpurun_out/prof_rn/*kernel_trace.csv 2>/dev/null | head -n 1)
python3 $R/scripts/step_breakdown.py "$f" > $R/gpurun_out/rn_breakdown_final.txt
head -n 12 $R/gpurun_out/rn_breakdown_final.txt
tail -n 1 $R/gpurun_out/rn_breakdown_final.txt
rm -rf $R/gpurun_out/prof_rn
