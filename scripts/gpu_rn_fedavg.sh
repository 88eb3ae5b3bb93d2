set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 240 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 30 --warmup 5 --async-steps 0 > gpurun_out/rn256_v5.log 2>&1 &&
timeout -k 10 240 python bench.py --model resnet18_cifar --batch-per-gpu 512 --steps 30 --warmup 5 --async-steps 0 > gpurun_out/rn512_v5.log 2>&1 &&
timeout -k 10 240 bash scripts/prof_model.sh rn5 10 --model resnet18_cifar --batch-per-gpu 256 --async-steps 0 > gpurun_out/prof_rn5.log 2>&1 &&
cd $R && timeout -k 10 240 python -m distriflow_amd.launch fedavg --model lenet5 --batch 1024 --rounds 20 --local-steps 50 > gpurun_out/fedavg_dev.log 2>&1
rc=$?
cd $R; tail -1 gpurun_out/rn256_v5.log; tail -1 gpurun_out/rn512_v5.log; head -25 gpurun_out/prof_summary_rn5.txt; tail -3 gpurun_out/fedavg_dev.log
exit $rc
