#!/usr/bin/env python3
"""Mean per-dispatch value of every counter in rocprofv3 --pmc csv output, per kernel.
    python3 tools/pmc_table.py gpurun_out/sq/sq1 [gpurun_out/sq/sq2 ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[row.get("Kernel_Name", "")[:40]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-22s %14.4g" % (c, sum(v) / len(v)))
