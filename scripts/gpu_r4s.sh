#!/usr/bin/env bash
# FedAvg (BASELINE config 5) on the device engine: 1 GPU, then a 4-process rehearsal sharing the GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 240 python -m distriflow_amd.launch fedavg --model lenet5 --batch 1024 --rounds 20 --local-steps 50 > gpurun_out/fedavg_1.log 2>&1 || { tail -n 20 gpurun_out/fedavg_1.log; exit 1; }
tail -n 1 gpurun_out/fedavg_1.log
DISTRIFLOW_BACKEND=gloo timeout -k 10 300 python -m distriflow_amd.launch --nproc 4 fedavg --model lenet5 --batch 1024 --rounds 10 --local-steps 20 > gpurun_out/fedavg_4.log 2>&1 || { tail -n 20 gpurun_out/fedavg_4.log; exit 1; }
tail -n 1 gpurun_out/fedavg_4.log
