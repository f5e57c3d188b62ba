#!/usr/bin/env python3
"""Device busy time of a rocprofv3 kernel trace: the union of kernel
intervals, per-kernel totals, and the idle gaps between them.
usage: trace_busy.py DIR [skip_first_ms]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
ev.sort()
if not ev:
    sys.exit("no kernels")
t0 = ev[0][0] + float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else ev[0][0]
ev = [e for e in ev if e[0] >= t0]
busy = 0
cur_s, cur_e = ev[0][0], ev[0][1]
gaps = []
per = defaultdict(lambda: [0, 0])
for s, e, n in ev:
    per[n][0] += 1
    per[n][1] += e - s
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = ev[-1][1] - ev[0][0]
print("span %.2f ms, busy %.2f ms (%.0f%%), %d kernels, %d gaps" % (span / 1e6, busy / 1e6, 100 * busy / span, len(ev), len(gaps)))
gaps.sort()
if gaps:
    q = lambda p: gaps[min(len(gaps) - 1, int(p * len(gaps)))] / 1e3
    print("gaps us: p10 %.1f p50 %.1f p90 %.1f max %.1f, sum %.2f ms" % (q(.1), q(.5), q(.9), gaps[-1] / 1e3, sum(gaps) / 1e6))
for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    print("  %-28s %6d launches %9.3f ms  avg %7.1f us" % (n, c, t / 1e6, t / c / 1e3))
