#!/usr/bin/env bash
# PMC passes over scripts/bench_convpool.py (plain conv vs pooled-epilogue conv), one run per pass
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmccp
rm -rf $O; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/t -o k --output-format csv -- python3 $R/scripts/bench_convpool.py 1024
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS -d $O/p1 -o k --output-format csv -- python3 $R/scripts/bench_convpool.py 1024
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p2 -o k --output-format csv -- python3 $R/scripts/bench_convpool.py 1024
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/p3 -o k --output-format csv -- python3 $R/scripts/bench_convpool.py 1024
python3 $R/scripts/pmc_summary.py $O/p1 $O/p2 $O/p3 > $O/summary.txt 2>&1 || true
cat $O/summary.txt
