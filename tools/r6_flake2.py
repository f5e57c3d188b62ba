"""Stress the deferred-output C2x64r parity case (GPU box), keeping the event
log of any stream whose digest differs from the reference's:
python tools/r6_flake2.py REPS OUTDIR"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden  # noqa: E402
import scenario_lib as S  # noqa: E402

reps, out = int(sys.argv[1]), sys.argv[2]
os.makedirs(out, exist_ok=True)
bad_runs = 0
for name, defer in (("C2x64r", 1), ("C2x64", 1), ("C2x64r", 8)):
    cfg = golden.config(name)
    want = golden.load(name)["digests"]
    for k in range(reps):
        # the harness dumps one stream's log per run: rotate through them
        idx = k % cfg.streams
        path = os.path.join(out, "%s_d%d_run%d_s%d.txt" % (name, defer, k, idx))
        os.environ["SCENARIO_DUMP"] = "%d:%s" % (idx, path)
        res, rep = S.run_batch(S.AMD_LIB, cfg, verify=True, defer=defer, threads=16,
                               groups=2 if cfg.streams >= 8 else 1)
        got = S.digests(res)
        bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
        if bad or rep.mismatches:
            bad_runs += 1
            print(name, defer, "run", k, "mismatches", rep.mismatches, "streams differ", bad[:8],
                  "dumped", idx, flush=True)
        elif os.path.exists(path):
            os.remove(path)
    print(name, "defer", defer, "done", flush=True)
print("bad runs", bad_runs, flush=True)
