#!/usr/bin/env bash
# Counter collection for the bench (run on the GPU box): two passes of SQ counters + one of LDS/TCC.
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3"}
rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc1 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc2 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
