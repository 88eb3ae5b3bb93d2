#!/usr/bin/env bash
# generic igemm gather change: kernel + engine tests, ResNet-18 bench, stem kernels in the breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_general_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r4r.log 2>&1 || { tail -n 30 gpurun_out/t_r4r.log; exit 1; }
tail -n 1 gpurun_out/t_r4r.log
for i in 1 2; do
timeout -k 10 200 python3 bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 100 --warmup 10 --async-steps 0 > gpurun_out/b_rn.json 2> gpurun_out/b_rn.err || { tail -n 20 gpurun_out/b_rn.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b_rn.json'));print('resnet18', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_rn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o k --output-format csv -- python3 $R/bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 20 --warmup 3 --async-steps 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_rn.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_rn -name '*kernel_trace.csv' | head -n 1)
python3 scripts/step_breakdown.py "$f" sgd_multi --order > gpurun_out/prof_rn.txt
grep "igemm_fwd\|igemm_wgrad\|total" gpurun_out/prof_rn.txt | head -n 5
