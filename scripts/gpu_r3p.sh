#!/usr/bin/env bash
# round-3 session P: conv3_halo one-step prefetch + split-K; wave-state counters of the halo kernels (layer 1, 2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
export DISTRIFLOW_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo or splitk" \
  > gpurun_out/t_p.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t_p.log | head -n 30; tail -n 30 gpurun_out/t_p.log; exit 1; }
tail -n 1 gpurun_out/t_p.log
timeout -k 10 200 python scripts/convbench.py > gpurun_out/cb_p.txt 2>&1 || { tail -n 20 gpurun_out/cb_p.txt; exit 1; }
cat gpurun_out/cb_p.txt
timeout -k 10 300 python bench.py --model resnet18_cifar --batch-per-gpu 256 --steps 100 --warmup 10 --async-steps 0 > gpurun_out/b_rn_p.log 2>&1 || { tail -n 20 gpurun_out/b_rn_p.log; exit 1; }
tail -n 1 gpurun_out/b_rn_p.log
cd /tmp && export TMPDIR=/tmp
for L in l1 l2; do
  rm -rf $R/gpurun_out/pmc_h_$L
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $R/gpurun_out/pmc_h_$L -o pmc --output-format csv -- python3 $R/scripts/convbench.py $L > $R/gpurun_out/pmc_h_$L.log 2>&1 || { tail -n 5 $R/gpurun_out/pmc_h_$L.log; exit 1; }
  rm -rf $R/gpurun_out/pmc_h2_$L
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_h2_$L -o pmc --output-format csv -- python3 $R/scripts/convbench.py $L > $R/gpurun_out/pmc_h2_$L.log 2>&1 || { tail -n 5 $R/gpurun_out/pmc_h2_$L.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_h_$L $R/gpurun_out/pmc_h2_$L > $R/gpurun_out/pmc_halo_$L.txt
done
cat $R/gpurun_out/pmc_halo_l1.txt $R/gpurun_out/pmc_halo_l2.txt
