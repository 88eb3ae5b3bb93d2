#!/usr/bin/env bash
# round-3 GPU session G: LeNet PMC passes (train + reduce), 2-rank rehearsal bench + per-rank step profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
bash scripts/pmc_lenet.sh > gpurun_out/pmc_lenet.log 2>&1 || { tail -n 20 gpurun_out/pmc_lenet.log; exit 1; }
grep -A 1 "lenet_" gpurun_out/pmc_lenet_summary.txt
cd "$R"
bash scripts/prof_ranks.sh 2 --steps 60 --warmup 5 --async-steps 0 > gpurun_out/prof_ranks.log 2>&1 || { tail -n 30 gpurun_out/prof_ranks.log; exit 1; }
cat gpurun_out/prof_ranks.log | grep -v "^W2026\|^E2026" | tail -n 20
