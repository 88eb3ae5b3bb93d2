#!/usr/bin/env bash
# reference CNN (model.json) B=1024: bench + kernel breakdown + khead phase stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --model keras_cnn --batch-per-gpu 1024 --steps 100 --warmup 10 > gpurun_out/b_kc.json 2> gpurun_out/b_kc.err || { tail -n 20 gpurun_out/b_kc.err; exit 1; }
cut -c1-400 gpurun_out/b_kc.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_kc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kc -o k --output-format csv -- python3 $R/bench.py --model keras_cnn --batch-per-gpu 1024 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_kc.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_kc.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_kc -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" kcnn_reduce > gpurun_out/prof_kc.txt
cat gpurun_out/prof_kc.txt
timeout -k 10 200 python3 scripts/kheadstamps.py > gpurun_out/kheadstamps.txt 2>&1 || { tail -n 20 gpurun_out/kheadstamps.txt; exit 1; }
head -n 14 gpurun_out/kheadstamps.txt
