#!/usr/bin/env bash
# Keras CNN conv block with packed conv1 FMAs: numerics (bit-exact vs per-layer path), bench x2, breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kcnn_fused_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4w.log 2>&1 || { tail -n 30 gpurun_out/t_r4w.log; exit 1; }
tail -n 1 gpurun_out/t_r4w.log
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --model keras_cnn --batch-per-gpu 1024 --steps 100 --warmup 10 > gpurun_out/b_kc.json 2> gpurun_out/b_kc.err || { tail -n 20 gpurun_out/b_kc.err; exit 1; }
  cut -c1-200 gpurun_out/b_kc.json
done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_kc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kc -o k --output-format csv -- python3 $R/bench.py --model keras_cnn --batch-per-gpu 1024 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_kc.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_kc.log; exit 1; }
f=$(ls $R/gpurun_out/prof_kc/*/*kernel_trace.csv $R/gpurun_out/prof_kc/*kernel_trace.csv 2>/dev/null | head -n 1)
python3 $R/scripts/step_breakdown.py "$f" > $R/gpurun_out/kc_breakdown.txt
cat $R/gpurun_out/kc_breakdown.txt
rm -rf $R/gpurun_out/prof_kc
