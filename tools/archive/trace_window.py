#!/usr/bin/env python3
"""Print the device events (kernels, copies) of a rocprofv3 CSV trace
directory between two host timestamps (ms, CLOCK_MONOTONIC, the clock of the
engine's SGPU_TIMELINE lines):  trace_window.py DIR T0_MS T1_MS"""
import csv
import glob
import sys

d, t0, t1 = sys.argv[1], float(sys.argv[2]) * 1e6, float(sys.argv[3]) * 1e6
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].split("(")[0], r["Grid_Size_X"]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"], ""))
ev.sort()
prev = None
for s, e, name, g in ev:
    if s < t0 or s > t1:
        continue
    gap = (s - prev) / 1e3 if prev else 0.0
    print("%14.3f  +%7.1f us  %7.1f us  %-40s %s" % (s / 1e6, gap, (e - s) / 1e3, name, g))
    prev = e
