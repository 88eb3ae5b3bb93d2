#!/usr/bin/env bash
# round-3 GPU session B: async PS fused path timing + kernel traces, callbacks tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_callbacks_gpu.py tests/test_async_ps_gpu.py > gpurun_out/t_cb.log 2>&1 || { tail -n 40 gpurun_out/t_cb.log; exit 1; }
tail -n 3 gpurun_out/t_cb.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > gpurun_out/b1.log 2>&1 || { cat gpurun_out/b1.log; exit 1; }
cat gpurun_out/b1.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_sync $R/gpurun_out/prof_async
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sync -o k --output-format csv -- python3 $R/bench.py --steps 60 --warmup 5 --async-steps 0 > $R/gpurun_out/prof_sync.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_sync.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_async -o k --output-format csv -- python3 $R/bench.py --mode async --steps 60 --warmup 5 > $R/gpurun_out/prof_async.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_async.log; exit 1; }
cd $R
for d in prof_sync prof_async; do
  f=$(find gpurun_out/$d -name '*kernel_trace.csv' | head -n 1)
  echo "== $d"; tail -n 1 gpurun_out/$d.log
  python3 scripts/step_breakdown.py "$f" lenet_reduce | tee gpurun_out/$d.txt
done
