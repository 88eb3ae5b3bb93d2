#!/usr/bin/env bash
# L2 / L1 / wave-state counters of the ResNet-18 conv kernels (scripts/convbench.py <layer>), one pass
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
L=${1:-l2}
rm -rf $R/gpurun_out/pmc_conv_$L
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD -d $R/gpurun_out/pmc_conv_$L -o pmc --output-format csv -- python3 $R/scripts/convbench.py $L
python3 - $R/gpurun_out/pmc_conv_$L <<'PY' > $R/gpurun_out/pmc_conv_$L.txt
import csv, glob, sys
from collections import defaultdict
v = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in v.items():
    print(k)
    print("   " + "  ".join(f"{n}={sum(x) / len(x):.4g}" for n, x in sorted(c.items())))
PY
cat $R/gpurun_out/pmc_conv_$L.txt
