#!/usr/bin/env bash
# round-3 session K (re-entry): whole GPU suite, headline bench, reference-CNN bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_full.log 2>&1 || { grep -E "FAILED|ERROR|Error|assert" gpurun_out/t_full.log | head -n 30; tail -n 30 gpurun_out/t_full.log; exit 1; }
tail -n 1 gpurun_out/t_full.log
timeout -k 10 200 python bench.py > gpurun_out/b_lenet.log 2>&1 || { tail -n 20 gpurun_out/b_lenet.log; exit 1; }
tail -n 1 gpurun_out/b_lenet.log
timeout -k 10 200 python bench.py --model keras_cnn --batch-per-gpu 1024 --steps 200 --warmup 20 --async-steps 0 > gpurun_out/b_kc.log 2>&1 || { tail -n 20 gpurun_out/b_kc.log; exit 1; }
tail -n 1 gpurun_out/b_kc.log
