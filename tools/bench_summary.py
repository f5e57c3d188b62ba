#!/usr/bin/env python3
"""One summary line of a bench.py JSON output: bench_summary.py LABEL LOG"""
import json
import sys

label, path = sys.argv[1], sys.argv[2]
line = [l for l in open(path).read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
dev, host = d["device"], d["host"]
print("%-8s value %8.1f GB/s  %6.3f ms/step  exec %.3f ms  device %.3f ms  frac %.4f  step %.2f flush %.2f"
      % (label, d["value"], d["ms_per_step"], dev["exec_ms_per_step"], dev["device_ms_per_step"],
         d["roofline"]["frac"], host["phase_ms_per_step"]["step"], host["phase_ms_per_step"]["flush"]))
