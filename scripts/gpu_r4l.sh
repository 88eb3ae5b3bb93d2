#!/usr/bin/env bash
# 8-rank rehearsal of the driver's N = 8 bench on one GPU (ranks share cuda:0, gloo control plane, the fused
# in-kernel exchange over IPC): checks the whole N > 1 path -- self-test at bind, two-launch step,
# JSON line -- not its speed (the 8 ranks time-slice one device)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
DISTRIFLOW_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 \
  bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/b_8r.log 2>&1 || { tail -n 40 gpurun_out/b_8r.log; exit 1; }
grep metric gpurun_out/b_8r.log | cut -c1-1200
