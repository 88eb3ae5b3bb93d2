#!/usr/bin/env bash
# Counter passes over a bench step (default: the fused LeNet-5 headline; extra args go to bench.py, e.g.
# --model keras_cnn --batch-per-gpu 1024).  Each pass has its own hard time limit; counters per block
# within the gfx950 slot limits.  Summaries: python3 scripts/pmc_summary.py gpurun_out/pmcl*
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
ARGS="--steps 10 --warmup 3 --async-steps 0 $*"
rm -rf $R/gpurun_out/pmcl1 $R/gpurun_out/pmcl2 $R/gpurun_out/pmcl3
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d $R/gpurun_out/pmcl1 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmcl2 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcl3 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmcl1 $R/gpurun_out/pmcl2 $R/gpurun_out/pmcl3 > $R/gpurun_out/pmc_lenet_summary.txt
cat $R/gpurun_out/pmc_lenet_summary.txt
