#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc CSV output (counter_collection.csv), merged over passes."""
import csv
import glob
import sys
from collections import defaultdict

dirs = sys.argv[1:] or ["gpurun_out/pmc1", "gpurun_out/pmc2"]
vals = defaultdict(lambda: defaultdict(list))
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void dfa::", "").replace("dfa::", "").replace("(anonymous namespace)::", "")[:72]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_MFMA",
        "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
        "SQ_VALU_MFMA_BUSY_CYCLES", "FETCH_SIZE", "WRITE_SIZE", "SQ_LDS_IDX_ACTIVE"]
for k, c in sorted(vals.items()):
    print(k)
    names = [n for n in cols if c.get(n)] + sorted(n for n in c if n not in cols)
    print("   " + "  ".join(f"{n.replace('SQ_', '')}={sum(c[n]) / len(c[n]):.3g}" for n in names))
