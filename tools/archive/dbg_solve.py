"""Debug aid: mismatches / failed streams of a few configs under the current
environment (run it under different SGPU_* / SIAMESE_AMD_* settings)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden  # noqa: E402
import scenario_lib as S  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else ""
for name, threads, groups, dge in [("C4x256", 16, 4, False), ("C2x64", 16, 2, False), ("C2h", 0, 2, False),
                                   ("C2h", 0, 2, True), ("C4x1024hr", 0, 4, False)]:
    cfg = golden.config(name)
    res, rep = S.run_batch(S.AMD_LIB, cfg, verify=True, threads=threads, groups=groups, device_ge=dge)
    want = golden.load(name)["digests"]
    bad = sum(1 for a, b in zip(S.digests(res), want) if a != b)
    print("%s %-10s dge=%d mismatches %d bad_streams %d status %s" % (tag, name, dge, rep.mismatches, bad,
                                                                      S.summary(res)["status"]), flush=True)
