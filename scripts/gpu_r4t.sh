#!/usr/bin/env bash
# LeNet-5 B=4096 per-kernel stats of the shipped step (rocprofv3 kernel trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/prof_ln
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ln -o k --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 > $R/gpurun_out/prof_ln.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_ln.log; exit 1; }
f=$(find $R/gpurun_out/prof_ln -name '*kernel_stats.csv' | head -n 1)
head -n 8 "$f" | cut -d, -f1-8
