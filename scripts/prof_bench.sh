#!/usr/bin/env bash
# rocprofv3 per-kernel stats of the headline bench (kernel trace only; counters are collected separately)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof
rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o k --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 "$@"
python3 $R/scripts/prof_summary.py $R/gpurun_out/prof 58 > $R/gpurun_out/prof_summary.txt
cat $R/gpurun_out/prof_summary.txt
