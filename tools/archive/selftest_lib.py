"""Solve-path self-test of a library variant (GPU box):
    python tools/selftest_lib.py siamese_amd/libsiamese_amd_X.so
Prints sgpu_selftest_solve_paths' result and stats for seeds 1..3, clean and
with inconsistent data (see tests/test_gpu_parity.py)."""
import ctypes
import sys

lib = ctypes.CDLL(sys.argv[1])
assert lib.sgpu_init(-1) == 0
ok = True
for corrupt in (0, 1):
    for seed in (1, 2, 3):
        st = (ctypes.c_uint32 * 4)()
        rc = lib.sgpu_selftest_solve_paths(ctypes.c_uint32(seed), ctypes.c_uint32(64), ctypes.c_uint32(corrupt), st)
        good = rc == 0 and st[0] == 0 and st[1] == 0 and (st[2] == 0 if not corrupt else 18 <= st[2] <= 22)
        ok &= good
        print("seed %d corrupt %d: rc %d diff tr %d mfma %d flagged tr %d mfma %d %s" %
              (seed, corrupt, rc, st[0], st[1], st[2], st[3], "ok" if good else "FAIL"))
sys.exit(0 if ok else 1)
