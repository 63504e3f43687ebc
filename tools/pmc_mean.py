#!/usr/bin/env python3
"""Mean per launch of every counter in a rocprofv3 --pmc CSV, for the kernels whose name contains
a filter (default "kkt_scan").  Usage: pmc_mean.py <run_counter_collection.csv> [filter]"""
import csv, json, sys
from collections import defaultdict

path = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "kkt_scan"
acc = defaultdict(list)
for r in csv.DictReader(open(path)):
    if kname in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: {"mean": sum(v) / len(v), "launches": len(v)} for k, v in sorted(acc.items())}))
