#!/usr/bin/env bash
# Keras CNN bench A/B of two builds of the extension (build_ab/_C_old.so vs _C_new.so), alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
for k in 1 2 3; do
  for v in old new; do
    cp build_ab/_C_$v.so distriflow_amd/_C.so
    timeout -k 10 200 python3 bench.py --model keras_cnn --batch-per-gpu 1024 --steps 100 --warmup 10 > gpurun_out/b_kc_ab.json 2> gpurun_out/b_kc_ab.err || { tail -n 20 gpurun_out/b_kc_ab.err; exit 1; }
    echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/b_kc_ab.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  done
done
cp build_ab/_C_new.so distriflow_amd/_C.so
