"""Manual GPU sanity run: drop-in API of libsiamese_amd vs the reference on
small versions of every workload.  Not collected by pytest."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import scenario_lib as S  # noqa: E402

cases = [
    ("C1", S.CONFIGS["C1"]),
    ("C1var", S.CONFIGS["C1var"]),
    ("C2x16", S.replace(S.CONFIGS["C2"], streams=16)),
    ("C4x16", S.replace(S.CONFIGS["C4"], streams=16)),
    ("C3x1500", S.replace(S.CONFIGS["C3"], originals=1500)),
]
if len(sys.argv) > 1 and sys.argv[1] == "big":
    cases += [("C3", S.CONFIGS["C3"]), ("C4x256", S.replace(S.CONFIGS["C4"], streams=256))]
bad_total = 0
for name, cfg in cases:
    ref, rs, rw = S.run_capi(S.REF_LIB, cfg, threads=1)
    t = time.time()
    amd, as_, aw = S.run_capi(S.AMD_LIB, cfg, threads=1)
    bad = [i for i in range(cfg.streams) if ref[i].digest != amd[i].digest or ref[i].status != amd[i].status]
    bad_total += len(bad)
    print("%-8s streams=%d mismatch=%d ref=%.3fs amd=%.3fs %s" % (name, cfg.streams, len(bad), rw, aw,
          S.summary(amd)), flush=True)
print("TOTAL MISMATCH", bad_total)
sys.exit(1 if bad_total else 0)
