#!/usr/bin/env python3
"""Per-barrier work and wait of k_exec's waves (profiling variant
tools/variants/exec_barriers.py): runs a short headline bench through the
variant library and prints, for each barrier in source order, the share of
all wave time spent working before it and waiting at it.
usage: python tools/barrier_clocks.py siamese_amd/libsiamese_amd_barriers.so [bench options]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

lib = sys.argv[1]
bench.main(["--library", lib, "--steps", "3", "--warmup", "1", "--no-cpu", "--no-e2e", "--no-legs",
            "--no-verify"] + sys.argv[2:])
L = ctypes.CDLL(os.path.abspath(lib))
out = (ctypes.c_ulonglong * 64)()
L.sgpu_debug_phase_clocks(out)
total = sum(out[k] + out[32 + k] for k in range(11)) or 1
names = {11: "version units", 12: "update units", 13: "plan units", 17: "planned-row quad tasks",
         19: "general rows"}
for k, cnt in ((11, 14), (12, 15), (13, 16), (17, 18), (19, 20)):
    if out[cnt]:
        print("%-24s %10d units, %8.0f clocks each, %5.1f%% of wave clocks" % (names[k], out[cnt], out[k] / out[cnt],
                                                                           100.0 * out[k] / max(1, sum(out[j] + out[32 + j] for j in range(11)))))
print("barrier  work%%   wait%%   (of all k_exec wave clocks, %.3g)" % total)
for k in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10):
    if out[k] or out[32 + k]:
        print("%5d   %6.1f  %6.1f" % (k, 100.0 * out[k] / total, 100.0 * out[32 + k] / total))
