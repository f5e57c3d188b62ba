"""Pipelined stream groups keep every byte intact (CPU backend double).

With several groups in flight, a buffer that one job's completed submission
released can be handed to another job's next submission.  The batch driver
must therefore read (gather) a completed job's packets before ANY further
submission is enqueued (include/siamese_gpu.h, device pointer lifetime).
C2's streaming decoder slides its window past delivered packets, so its
recovered packets are released as soon as they are delivered: before the
fix, 1024 C2 streams in 4 groups produced byte mismatches on 3 streams."""
import scenario_lib as S


def test_c2_four_groups_bytes_verified():
    cfg = S.replace(S.CONFIGS["C2"], hash_data=0, streams=1024)
    sess = S.BatchSession(S.SIM_LIB, cfg)
    try:
        res, rep = sess.run(steps=0, warmup=1, verify=True, threads=8, groups=4)
        assert rep.checked > 0
        assert rep.mismatches == 0
        assert not any(r.status for r in res), S.summary(res)["status"]
    finally:
        sess.close()


def test_oplincombs_batches_match_plain_ops():
    """OP_LINCOMBS (independent combinations dealt to whole waves) gives the
    same bytes as one plain op per combination: C2's Cauchy rows and
    eliminations, digests from both runs equal."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import scenario_lib as S\n"
        "cfg = S.replace(S.CONFIGS['C2'], streams=64)\n"
        "res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, threads=4)\n"
        "assert rep.mismatches == 0 and not any(r.status for r in res)\n"
        "print(S.digests(res))\n" % os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for v in ("0", "1"):
        env = dict(os.environ, SIAMESE_AMD_LC_BATCH=v)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[v] = r.stdout.strip().splitlines()[-1]
    assert out["0"] == out["1"]
