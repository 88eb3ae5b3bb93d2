#!/usr/bin/env bash
# round-3 session S: ResNet whole-model gradient cosines (tightening the bound), 2-rank LeNet-5 bench rehearsal
# on one GPU (LL self-test + fused exchange), reference-CNN step breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "model_gradients_match_cpu" \
  > gpurun_out/t_s.log 2>&1 || { tail -n 30 gpurun_out/t_s.log; exit 1; }
grep -E "^(resnet18_cifar|lenet5|keras_cnn|mlp_mnist) " gpurun_out/t_s.log | cut -c1-3000
tail -n 1 gpurun_out/t_s.log
DISTRIFLOW_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/b_2r.log 2>&1 || { tail -n 30 gpurun_out/b_2r.log; exit 1; }
grep metric gpurun_out/b_2r.log | cut -c1-700
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_kc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kc -o k --output-format csv -- python3 $R/bench.py --model keras_cnn --batch-per-gpu 1024 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_kc.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_kc.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_kc -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" kcnn_reduce > gpurun_out/prof_kc.txt
cat gpurun_out/prof_kc.txt
