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


def test_paired_ingest_matches_separate_ingest():
    """Two-destination ingest descriptors (an encoder and then its decoder
    taking in one device original) give the digests of separate ingests, and
    the reference's (golden C4x256), with every recovered byte verified."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import scenario_lib as S, golden\n"
        "res, rep = S.run_batch(S.SIM_LIB, golden.config('C4x256'), verify=True, threads=4, groups=2)\n"
        "assert rep.mismatches == 0 and not any(r.status for r in res)\n"
        "assert S.digests(res) == golden.load('C4x256')['digests']\n"
        "print(S.engine_dict(rep)['ingests'])\n" % os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for v in ("0", "1"):
        env = dict(os.environ, SIAMESE_AMD_INGEST_PAIRS=v)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[v] = int(r.stdout.strip().splitlines()[-1])
    assert out["1"] < out["0"]   # the pairs did form (fewer descriptors)


def test_pipelined_steps_keep_their_own_results():
    """Steps of one session may be in flight together (the next step's first
    job starts while the last one runs), and they run the same streams: each
    job keeps its own per-stream results, so the results describe exactly one
    run and the report counts every step's payload once."""
    cfg = S.replace(S.CONFIGS["C3"], hash_data=0, originals=600)
    sess = S.BatchSession(S.SIM_LIB, cfg)
    try:
        res1, rep1 = sess.run(steps=1, warmup=0, verify=False, groups=1, digest=False)
        one = sum(r.payload_bytes for r in res1)
        assert one == 600 * 1400
        assert rep1.payload_bytes == one
        res, rep = sess.run(steps=2, warmup=0, verify=False, groups=1, digest=False)
        assert sum(r.payload_bytes for r in res) == one
        assert rep.payload_bytes == 2 * one
        assert [r.encodes for r in res] == [r.encodes for r in res1]
    finally:
        sess.close()


def test_released_buffers_wait_for_the_published_ticket():
    """A completed submission's released buffers are filed in the depot just
    before its ticket is published; with that window widened (the completer
    sleeps between the two), no stream may hand such a buffer to a new
    submission before the harness has gathered the completed job's outputs:
    every recovered byte of 1024 C2 streams in 4 pipelined groups verifies."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import scenario_lib as S\n"
        "cfg = S.replace(S.CONFIGS['C2'], hash_data=0, streams=1024)\n"
        "sess = S.BatchSession(S.SIM_LIB, cfg)\n"
        "res, rep = sess.run(steps=0, warmup=1, verify=True, threads=8, groups=4)\n"
        "sess.close()\n"
        "assert rep.checked > 0 and rep.mismatches == 0, rep.mismatches\n"
        "assert not any(r.status for r in res)\n"
        "print('ok', rep.checked)\n" % os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SGPU_TEST_PUBLISH_DELAY_US="300")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().startswith("ok")


def test_merged_rounds_match_separate_rounds():
    """A job's later rounds ride in the next new job's fork-join and
    submission (the default) or each take their own (SCENARIO_MERGE_ROUNDS=0):
    the golden C4x256 digests of the reference either way, with the chained
    device decode (its second round is the decode's finish), 8 groups over 2
    steps (jobs of both steps in flight together), every recovered byte
    verified; merged, the run takes fewer submissions."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import scenario_lib as S, golden\n"
        "sess = S.BatchSession(S.SIM_LIB, golden.config('C4x256'))\n"
        "res, rep = sess.run(steps=0, warmup=1, verify=True, threads=4, groups=8, device_ge=True)\n"
        "assert rep.mismatches == 0 and not any(r.status for r in res)\n"
        "assert S.digests(res) == golden.load('C4x256')['digests']\n"
        "res2, rep2 = sess.run(steps=2, warmup=0, verify=False, threads=4, groups=8, digest=False,\n"
        "                      device_ge=True)\n"
        "assert not any(r.status for r in res2)\n"
        "sess.close()\n"
        "print(rep2.rounds)\n" % os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for v in ("0", "1"):
        env = dict(os.environ, SCENARIO_MERGE_ROUNDS=v)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[v] = int(r.stdout.strip().splitlines()[-1])
    assert out["1"] < out["0"]   # the later rounds did ride along
