#!/usr/bin/env bash
# rocprofv3 per-kernel table of the headline bench (kernel trace only; counters are collected separately).
# MARKER: a kernel launched once per timed step of the measured engine (default: the LeNet-5 sync reduce);
# scripts/prof_summary.py takes the steady-state steps between its launches (no hand-given step count).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
MARKER=${MARKER:-lenet_reduce_kernel<0>}
OUT=${OUT:-prof}
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/$OUT
rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$OUT -o k --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 "$@"
python3 $R/scripts/prof_summary.py $R/gpurun_out/$OUT --marker "$MARKER" > $R/gpurun_out/${OUT}_summary.txt
cat $R/gpurun_out/${OUT}_summary.txt
