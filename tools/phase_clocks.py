#!/usr/bin/env python3
"""Per-phase shader clocks of k_exec's OP_ROWS path (profiling build:
tools/build_variant.sh phase -DSGPU_PHASE_CLOCKS).  Runs a short C4 bench
through the variant library, then prints the clocks per workgroup-op.
usage: python tools/phase_clocks.py siamese_amd/libsiamese_amd_phase.so [bench options]"""
import ctypes
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

lib = sys.argv[1]
if len(sys.argv) > 2 and sys.argv[2] in ("C2", "C3", "C5"):
    # a leg instead of the headline: python tools/phase_clocks.py LIB C3
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import scenario_lib as S  # noqa: E402
    cfg = S.replace(S.CONFIGS[sys.argv[2]], hash_data=0)
    sess = S.BatchSession(lib, cfg, device=0)
    try:
        sess.run(steps=1, warmup=0, verify=False, threads=0, groups=2 if sys.argv[2] == "C2" else 1,
                 digest=False, defer=4 if sys.argv[2] == "C2" else 8)
    finally:
        sess.close()
else:
    bench.main(["--library", lib, "--steps", "3", "--warmup", "1", "--no-cpu", "--no-e2e", "--no-legs"] + sys.argv[2:])
L = ctypes.CDLL(os.path.abspath(lib))
out = (ctypes.c_ulonglong * 64)()
L.sgpu_debug_phase_clocks(out)
ops = max(1, out[8])
names = ["block load", "stage+plan", "sum updates", "stage sums", "sums barrier", "rows"]
print("OP_ROWS workgroup-ops %d, rows %.1f, updates %.1f, window %.1f, staged %.1f per op"
      % (out[8], out[9] / ops, out[10] / ops, out[11] / ops, out[12] / ops))
for k, nm in enumerate(names):
    print("  %-14s %10.0f clocks per op" % (nm, out[k] / ops))
print("  rows detail (wave 0 quad tasks): descriptors %.0f, terms %.0f, stores %.0f clocks per op"
      % (out[13] / ops, out[14] / ops, out[15] / ops))
print("  detail (wave 0): update units %.0f, plan pairs %.0f clocks per op; stage re-read in %.1f%% of ops"
      % (out[19] / ops, out[20] / ops, 100.0 * out[21] / ops))
print("kernel: %d workgroups, %.0f clocks each" % (out[7], out[6] / max(1, out[7])))
wgs = max(1, out[7])
print("setup %.0f clocks per workgroup" % (out[32] / wgs))
for k, nm in enumerate(["LINCOMB", "LITERAL", "ROWS", "COPIES", "LINCOMBS"]):
    c = out[38 + k]
    print("  %-9s %8d ops, %10.0f clocks per op, %10.0f clocks per workgroup" % (
        nm, c, out[33 + k] / max(1, c), out[33 + k] / wgs))
print("OP_ROWS: thread 0 waits %.0f clocks per op at the op's closing barrier (other waves still in the rows phase)"
      % (out[43] / max(1, out[40])))
if out[46]:
    big = out[47]
    print("k_solve_prefix: setup %.0f, solve %.0f clocks per row (summed over solves); slowest wave %d clocks (m=%d)"
          % (out[44] / out[46], out[45] / out[46], big >> 8, big & 0xff))
    low = out[48] - out[49]
    print("  lower sweep %.0f, back-substitution %.0f clocks per row" % (low / out[46], (out[45] - low) / out[46]))
