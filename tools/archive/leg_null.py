"""Host control plane alone on one BASELINE config: the batch driver over
tools/libsiamese_null.so (no symbol work, no device), so the host share of a
leg can be timed on the GPU box's own cores.
usage: python tools/leg_null.py C2 [runs] [groups] [defer] [threads]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenario_lib as S  # noqa: E402


def main():
    name = sys.argv[1]
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    groups = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    defer = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    thr = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    cfg = S.replace(S.CONFIGS[name], hash_data=0)
    sess = S.BatchSession(os.path.join(ROOT, "tools", "libsiamese_null.so"), cfg, device=-1)
    try:
        sess.run(steps=0, warmup=1, verify=False, threads=thr, groups=groups, defer=defer)
        secs = []
        for _ in range(runs):
            res, rep = sess.run(steps=1, warmup=0, verify=False, threads=thr, groups=groups,
                                digest=False, defer=defer)
            secs.append(rep.seconds * 1e3)
    finally:
        sess.close()
    print("null %s groups %d defer %d threads %d ms/run %s rounds %d phases(last) %s" % (
        name, groups, defer, thr, [round(x, 2) for x in secs], rep.rounds,
        [round(x * 1e3, 2) for x in rep.phase_seconds]))


if __name__ == "__main__":
    main()
