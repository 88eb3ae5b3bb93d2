#!/usr/bin/env bash
# PMC counters of one fused conv+pool forward configuration (scripts/cpbench.py --only ...)
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
ONLY=${ONLY:-conv1}
for MASK in ${MASKS:-0 15}; do
  rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $R/gpurun_out/pmccp_${ONLY}_${MASK}_a -o pmc --output-format csv -- python3 $R/scripts/cpbench.py --only $ONLY --mask $MASK
  rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_BRANCH SQ_WAIT_INST_ANY -d $R/gpurun_out/pmccp_${ONLY}_${MASK}_b -o pmc --output-format csv -- python3 $R/scripts/cpbench.py --only $ONLY --mask $MASK
done
