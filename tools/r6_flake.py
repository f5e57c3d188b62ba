"""Repeat one deferred-output parity case and count digest mismatches
(GPU box): python tools/r6_flake.py NAME DEFER REPS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden  # noqa: E402
import scenario_lib as S  # noqa: E402

name, defer, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cfg = golden.config(name)
want = golden.load(name)["digests"]
bad_runs = 0
for k in range(reps):
    res, rep = S.run_batch(S.AMD_LIB, cfg, verify=True, defer=defer, threads=16,
                           groups=2 if cfg.streams >= 8 else 1)
    got = S.digests(res)
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    if bad or rep.mismatches:
        bad_runs += 1
        print("run", k, "mismatches", rep.mismatches, "streams differ", bad[:8], flush=True)
print(name, "defer", defer, "bad runs", bad_runs, "of", reps, flush=True)
