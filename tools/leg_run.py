"""Run one BASELINE config through the batch driver (for rocprofv3 traces of a
single leg):  python tools/leg_run.py C3 [runs] [groups]
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
    cfg = S.replace(S.CONFIGS[name], hash_data=0)
    lib = os.environ.get("SGPU_LIB", os.path.join(ROOT, "siamese_amd", "libsiamese_amd.so"))
    sess = S.BatchSession(lib, cfg, device=0 if "null" not in lib else -1)
    try:
        sess.run(steps=0, warmup=1, verify=False, threads=0, groups=groups)
        res, rep = sess.run(steps=runs, warmup=0, verify=False, threads=0, groups=groups, digest=False)
    finally:
        sess.close()
    if any(r.status for r in res):
        raise SystemExit("leg %s failed" % name)
    ph = [round(x / runs * 1e3, 3) for x in rep.phase_seconds]
    print("%s groups %d ms/run %.3f device %.3f rounds %.1f phases %s" % (
        name, groups, rep.seconds / runs * 1e3, rep.device_ms / runs, rep.rounds / runs, ph))


if __name__ == "__main__":
    main()
