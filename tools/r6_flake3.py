"""Repeat the GPU suite's deferred-output sequence in one process (GPU box):
the end-to-end pipelined cases, then every deferred case, REPS times.
python tools/r6_flake3.py REPS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import test_gpu_parity as T  # noqa: E402

reps = int(sys.argv[1])
fails = []
for r in range(reps):
    for name in ("C4x256", "C2x64"):
        try:
            T.test_batch_api_end_to_end_pipelined(name)
        except AssertionError as e:
            fails.append(("e2e", name, r, str(e)[:200]))
    for defer in (1, 8):
        for name in T.SMALL + ["C3", "C4x256", "C5x2000"]:
            try:
                T.test_batch_api_deferred_outputs(name, defer)
            except AssertionError as e:
                fails.append(("deferred", name, defer, r, str(e)[:200]))
                print("FAIL", fails[-1], flush=True)
    print("rep", r, "fails so far", len(fails), flush=True)
print("total fails", len(fails), fails, flush=True)
