#!/usr/bin/env bash
# PMC counters per kernel for any bench config (run on the GPU box), one rocprofv3 pass per counter
# group, each under its own hard time limit:  scripts/pmc_model.sh <tag> <bench args...>
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
rm -rf $R/gpurun_out/pmc_${TAG}_*
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_${TAG}_1 -o pmc --output-format csv -- python3 $R/bench.py "$@"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc_${TAG}_2 -o pmc --output-format csv -- python3 $R/bench.py "$@"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES FETCH_SIZE -d $R/gpurun_out/pmc_${TAG}_3 -o pmc --output-format csv -- python3 $R/bench.py "$@" || echo "pass 3 failed (counter unavailable?)"
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_${TAG}_1 $R/gpurun_out/pmc_${TAG}_2 $R/gpurun_out/pmc_${TAG}_3 > $R/gpurun_out/pmc_summary_${TAG}.txt
head -60 $R/gpurun_out/pmc_summary_${TAG}.txt
