"""Regenerate the golden fixtures from the upstream reference.

Runs only where oracle/_ref/libsiamese_ref.so exists (it is compiled from
/root/reference by oracle/Makefile).  Usage: python tests/golden/make_golden.py [name ...]
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import golden  # noqa: E402
import scenario_lib as S  # noqa: E402


def main(names):
    if not os.path.exists(S.REF_LIB):
        sys.exit("oracle/_ref/libsiamese_ref.so missing: run make -C oracle")
    for name in names or list(golden.FIXTURES):
        cfg = golden.config(name)
        t0 = time.time()
        res, _, wall = S.run_capi(S.REF_LIB, cfg, threads=min(8, cfg.streams))
        golden.save(name, cfg, res, wall)
        print("%-16s streams=%-5d %.2fs %s" % (name, cfg.streams, time.time() - t0,
                                               S.summary(res)), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
