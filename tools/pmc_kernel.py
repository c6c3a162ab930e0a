#!/usr/bin/env python3
"""Mean value per launch of every counter collected for kernels matching a name pattern.

    python tools/pmc_kernel.py <pattern> <run_dir> [<run_dir> ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

pat = sys.argv[1]
vals = defaultdict(list)
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                per[(r["Counter_Name"], r.get("Dispatch_Id", ""))] += float(r["Counter_Value"])
        for (name, _), v in per.items():
            vals[name].append(v)
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(vals.items())}, indent=1))
