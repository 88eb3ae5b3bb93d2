#!/usr/bin/env bash
# round-3 session W (final): whole GPU suite, smoke, headline bench, reference-CNN and ResNet-18 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_final.log 2>&1 || { grep -E "FAILED|ERROR|Error|assert" gpurun_out/t_final.log | head -n 30; tail -n 30 gpurun_out/t_final.log; exit 1; }
tail -n 1 gpurun_out/t_final.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 20 gpurun_out/smoke.log; exit 1; }
tail -n 2 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/b_final_k20.log 2>&1 || { tail -n 20 gpurun_out/b_final_k20.log; exit 1; }
tail -n 1 gpurun_out/b_final_k20.log | cut -c1-300
timeout -k 10 200 python bench.py > gpurun_out/b_final.log 2>&1 || { tail -n 20 gpurun_out/b_final.log; exit 1; }
tail -n 1 gpurun_out/b_final.log | cut -c1-300
timeout -k 10 200 python bench.py --model keras_cnn --batch-per-gpu 1024 --steps 200 --warmup 20 --async-steps 0 > gpurun_out/b_final_kc.log 2>&1 || { tail -n 20 gpurun_out/b_final_kc.log; exit 1; }
tail -n 1 gpurun_out/b_final_kc.log | cut -c1-200
timeout -k 10 200 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 200 --warmup 10 --async-steps 0 > gpurun_out/b_final_rn.log 2>&1 || { tail -n 20 gpurun_out/b_final_rn.log; exit 1; }
tail -n 1 gpurun_out/b_final_rn.log | cut -c1-200
