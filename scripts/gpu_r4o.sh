#!/usr/bin/env bash
# kernel-argument placement A/B: reduce-launch stamps and bench with / without HIP_FORCE_DEV_KERNARG=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python3 scripts/lenetstamps.py 4096 step > gpurun_out/ka_$v.txt 2>&1 || { tail -n 20 gpurun_out/ka_$v.txt; exit 1; }
  echo "HIP_FORCE_DEV_KERNARG=$v: $(grep 'both launches' gpurun_out/ka_$v.txt)"
  grep "launch span" gpurun_out/ka_$v.txt | head -n 2 | cut -c1-160
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --async-steps 0 > gpurun_out/ka_b$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ka_b$v.json'));print('  bench', d['value'], d['ms_per_step'])"
done
