#!/usr/bin/env bash
# LeNet phase-G change: numerics tests, stamps (train + reduce), bench K=20 / K=200, then the 8-rank
# rehearsal of the driver's N = 8 bench on one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
F="amdgpu.ids\|Gloo\|socket.cpp"
timeout -k 10 300 python -u -m pytest tests/test_lenet_fused_gpu.py tests/test_fused_dp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4m.log 2>&1 || { tail -n 30 gpurun_out/t_r4m.log; exit 1; }
tail -n 1 gpurun_out/t_r4m.log
timeout -k 10 200 python -u scripts/lenetstamps.py 4096 step 2>&1 | grep -v "$F" | tee gpurun_out/lenetstamps_r4m.txt
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r4m_k20.json 2> gpurun_out/b_r4m_k20.err || { tail -n 20 gpurun_out/b_r4m_k20.err; exit 1; }
cut -c1-300 gpurun_out/b_r4m_k20.json
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > gpurun_out/b_r4m_k200.json 2> gpurun_out/b_r4m_k200.err || { tail -n 20 gpurun_out/b_r4m_k200.err; exit 1; }
cut -c1-300 gpurun_out/b_r4m_k200.json
bash scripts/gpu_r4l.sh
