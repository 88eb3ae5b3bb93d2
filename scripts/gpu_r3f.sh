#!/usr/bin/env bash
# round-3 GPU session F: fused LeNet step correctness + bench + step profile + reduce stamps + kernarg probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_lenet_fused_gpu.py \
  tests/test_callbacks_gpu.py tests/test_async_ps_gpu.py tests/test_fused_dp_gpu.py > gpurun_out/t_f.log 2>&1 \
  || { grep -E "FAILED|Error" gpurun_out/t_f.log | head -n 30; tail -n 30 gpurun_out/t_f.log; exit 1; }
tail -n 3 gpurun_out/t_f.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/b1.log 2>&1 || { cat gpurun_out/b1.log; exit 1; }
cat gpurun_out/b1.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_sync
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sync -o k --output-format csv -- python3 $R/bench.py --steps 60 --warmup 5 --async-steps 0 > $R/gpurun_out/prof_sync.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_sync.log; exit 1; }
rm -rf $R/gpurun_out/prof_async
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_async -o k --output-format csv -- python3 $R/bench.py --mode async --steps 60 --warmup 5 > $R/gpurun_out/prof_async.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_async.log; exit 1; }
cd $R
for d in prof_sync prof_async; do
  f=$(find gpurun_out/$d -name '*kernel_trace.csv' | head -n 1)
  echo "== $d"
  python3 scripts/step_breakdown.py "$f" lenet_reduce | tee gpurun_out/$d.txt
done
timeout -k 10 200 python scripts/lenetstamps.py 4096 step > gpurun_out/stamps.log 2>&1 || { tail -n 30 gpurun_out/stamps.log; exit 1; }
grep -A 14 "dense  jobs" gpurun_out/stamps.log
