"""C2 verification under stream groups / gather modes (GPU box debugging aid):
    python tools/c2_debug.py STREAMS GROUPS"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenario_lib as S  # noqa: E402
S.SCENARIO_LIB = os.environ.get("SCENARIO_LIB", S.SCENARIO_LIB)

streams, groups = int(sys.argv[1]), int(sys.argv[2])
cfg = S.replace(S.CONFIGS["C2"], hash_data=0, streams=streams)
lib = os.environ.get("SGPU_LIB", os.path.join(ROOT, "siamese_amd", "libsiamese_amd.so"))
sess = S.BatchSession(lib, cfg, device=0)
res, rep = sess.run(steps=0, warmup=1, verify=True, threads=0, groups=groups)
bad = [i for i, r in enumerate(res) if r.status]
print("%s streams %d groups %d sync %s: mismatches %d checked %d bad streams %d %s" % (
    os.path.basename(lib), streams, groups, os.environ.get("SCENARIO_SYNC_GATHER"), rep.mismatches, rep.checked, len(bad),
    S.summary(res)["status"] if bad else ""), flush=True)
sess.close()
