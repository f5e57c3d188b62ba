"""Run one BASELINE config through the batch driver (for rocprofv3 traces of a
single leg):  python tools/leg_run.py C3 [runs] [groups] [defer]
Prints ms per run, device ms per run and rounds per run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenario_lib as S  # noqa: E402


def main():
    name = sys.argv[1]
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    groups = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    defer = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    base, _, count = name.partition("x")   # e.g. C4x1024: the first 1024 streams of C4
    cfg = S.replace(S.CONFIGS[base], hash_data=0)
    if count:
        cfg = S.replace(cfg, streams=int(count))
    lib = os.environ.get("SGPU_LIB", os.path.join(ROOT, "siamese_amd", "libsiamese_amd.so"))
    sess = S.BatchSession(lib, cfg, device=0 if "null" not in lib else -1)
    try:
        res0, rep0 = sess.run(steps=0, warmup=1, verify=True, threads=0, groups=groups, defer=defer)
        if rep0.mismatches or any(r.status for r in res0):
            raise SystemExit("leg %s: verification failed" % name)
        secs = []
        for _ in range(runs):
            res, rep = sess.run(steps=1, warmup=0, verify=False, threads=0, groups=groups, digest=False,
                                defer=defer, timing=os.environ.get("LEG_TIMING", "0") == "1")
            secs.append(rep.seconds * 1e3)
    finally:
        sess.close()
    if any(r.status for r in res):
        raise SystemExit("leg %s failed" % name)
    ph = [round(x * 1e3, 3) for x in rep.phase_seconds]
    print("%s groups %d defer %d ms/run %s device %.3f rounds %d phases(last) %s" % (
        name, groups, defer, [round(x, 2) for x in secs], rep.device_ms, rep.rounds, ph))


if __name__ == "__main__":
    main()
