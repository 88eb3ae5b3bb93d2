#!/usr/bin/env bash
# LeNet-5 B=4096 step time vs convpool persistent-grid sizing (DISTRIFLOW_DIAG cp_wpc / cp_minimgs)
set -o pipefail
out=gpurun_out/cp_sweep.log
: > $out
for cfg in "8 1" "4 1" "2 1" "8 2" "8 4" "8 8" "4 4"; do
  set -- $cfg
  echo "wpc=$1 minimgs=$2" >> $out
  DISTRIFLOW_DIAG=cp_wpc=$1,cp_minimgs=$2 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --async-steps 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $out || exit $?
done
cat $out
