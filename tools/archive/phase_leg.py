#!/usr/bin/env python3
"""Per-phase shader clocks of k_exec's OP_ROWS path over one leg run
(profiling build: tools/build_variant.sh phase -DSGPU_PHASE_CLOCKS).
usage: python tools/phase_leg.py siamese_amd/libsiamese_amd_phase.so C3 [groups] [defer]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenario_lib as S  # noqa: E402

lib, name = sys.argv[1], sys.argv[2]
groups = int(sys.argv[3]) if len(sys.argv) > 3 else 1
defer = int(sys.argv[4]) if len(sys.argv) > 4 else 0
cfg = S.replace(S.CONFIGS[name], hash_data=0)
sess = S.BatchSession(lib, cfg, device=0)
res, rep = sess.run(steps=1, warmup=0, verify=False, groups=groups, digest=False, defer=defer)
sess.close()
L = ctypes.CDLL(os.path.abspath(lib))
out = (ctypes.c_ulonglong * 64)()
L.sgpu_debug_phase_clocks(out)
ops = max(1, out[8])
names = ["block load", "stage+plan", "sum updates", "stage sums", "sums barrier", "rows"]
print("%s: %.1f ms, OP_ROWS workgroup-ops %d, rows %.1f, updates %.1f, window %.1f, staged %.1f per op"
      % (name, rep.seconds * 1e3, out[8], out[9] / ops, out[10] / ops, out[11] / ops, out[12] / ops))
for k, nm in enumerate(names):
    print("  %-14s %10.0f clocks per op" % (nm, out[k] / ops))
print("  rows detail (wave 0 quad tasks): descriptors %.0f, terms %.0f, stores %.0f clocks per op"
      % (out[13] / ops, out[14] / ops, out[15] / ops))
print("  versions: %.0f clocks per op, %d quad tasks with corrections" % (out[16] / ops, out[17]))
print("  version element iterations (lane 0 of each wave): %d combined, %d part-lane" % (out[24], out[25]))
print("  phase A on wave 0: before units %.0f, units %.0f, barrier %.0f clocks per op" % (out[30] / ops, out[31] / ops, out[2] / ops))
print("  phase A units (all waves): updates %d x %.0f clocks, plans %d x %.0f, versions %d x %.0f"
      % (out[27], out[19] / max(1, out[27]), out[28], out[20] / max(1, out[28]), out[29], out[26] / max(1, out[29])))
print("  general rows: terms %.0f, stores %.0f clocks per op, %d row units" % (out[18] / ops, out[22] / ops, out[23]))
print("kernel: %d workgroups, %.0f clocks each" % (out[7], out[6] / max(1, out[7])))
