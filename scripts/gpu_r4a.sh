#!/usr/bin/env bash
# round-4: the sharded lock-free PS + fused exchange self-test first, then the whole GPU suite, then the
# driver-style bench (sync + async)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_async_ps_gpu.py tests/test_fused_dp_gpu.py -x -v --timeout 420 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_r4a_ps.log 2>&1 || { tail -n 60 gpurun_out/t_r4a_ps.log; exit 1; }
tail -n 3 gpurun_out/t_r4a_ps.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r4a_k20.json 2> gpurun_out/b_r4a_k20.err || { tail -n 20 gpurun_out/b_r4a_k20.err; exit 1; }
cat gpurun_out/b_r4a_k20.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 420 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_async_ps_gpu.py --deselect tests/test_fused_dp_gpu.py > gpurun_out/t_r4a.log 2>&1 || { tail -n 40 gpurun_out/t_r4a.log; exit 1; }
tail -n 3 gpurun_out/t_r4a.log
