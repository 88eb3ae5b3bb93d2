#!/usr/bin/env bash
# rocprofv3 per-kernel stats of bench.py for any model:  scripts/prof_model.sh <tag> <steps> <bench args...>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; STEPS=$2; shift 2
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_$TAG
rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o k --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 3 "$@"
python3 $R/scripts/prof_summary.py $R/gpurun_out/prof_$TAG $((STEPS + 3)) > $R/gpurun_out/prof_summary_$TAG.txt
head -40 $R/gpurun_out/prof_summary_$TAG.txt
