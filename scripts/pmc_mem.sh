#!/usr/bin/env bash
# Memory-hierarchy counter passes over the bench step (L2 hit/miss, fabric read requests, L1->L2 reads).
# Summaries: python3 scripts/pmc_summary.py gpurun_out/pmcm*
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
ARGS="--steps 10 --warmup 3 --async-steps 0 $*"
rm -rf $R/gpurun_out/pmcm1 $R/gpurun_out/pmcm2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $R/gpurun_out/pmcm1 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE TA_BUSY_avr TA_TA_BUSY_sum -d $R/gpurun_out/pmcm2 -o pmc --output-format csv -- python3 $R/bench.py $ARGS
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmcm1 $R/gpurun_out/pmcm2 > $R/gpurun_out/pmc_mem_summary.txt
cat $R/gpurun_out/pmc_mem_summary.txt
