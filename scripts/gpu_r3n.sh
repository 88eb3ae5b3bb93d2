#!/usr/bin/env bash
# round-3 session N: two-group halo wgrad, ResNet-18 step breakdown with the halo kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" \
  > gpurun_out/t_n.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_n.log | head -n 30; tail -n 30 gpurun_out/t_n.log; exit 1; }
tail -n 1 gpurun_out/t_n.log
timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_n.txt 2>&1 || { tail -n 20 gpurun_out/cb_n.txt; exit 1; }
cat gpurun_out/cb_n.txt
for g in 1; do
  DISTRIFLOW_DIAG=halo_groups=$g timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_g$g.txt 2>&1 || { tail -n 20 gpurun_out/cb_g$g.txt; exit 1; }
  echo "halo_groups=$g"; grep -o "wgrad.*" gpurun_out/cb_g$g.txt
done
timeout -k 10 300 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 50 --warmup 10 --async-steps 0 > gpurun_out/b_rn_n.log 2>&1 || { tail -n 20 gpurun_out/b_rn_n.log; exit 1; }
tail -n 1 gpurun_out/b_rn_n.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_rn -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi > gpurun_out/prof_rn.txt
cat gpurun_out/prof_rn.txt
