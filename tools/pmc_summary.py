#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc CSVs: pmc_summary.py A.csv [B.csv ...]"""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    print(k)
    for c in sorted(acc[k]):
        v = acc[k][c]
        print("   %-24s %16.0f  (n=%d)" % (c, sum(v) / len(v), len(v)))
