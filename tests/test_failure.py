"""A device failure is sticky: once a flush's synchronisation fails, nothing
of that flush is delivered and every later call on every instance returns
Siamese_Disabled (the reference's EmergencyDisabled, siamese.h:147-150;
SiameseEncoder.cpp / SiameseDecoder.cpp set it and never clear it).

The fault is injected into the CPU test double of the backend
(HOSTSIM_FAIL_SYNC=N fails the N-th device synchronisation and all later
ones), in a child process because the failed engine is process-wide.
"""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent(r"""
    import ctypes, json, sys
    sys.path.insert(0, %(root)r)
    from siamese_amd.binding import SiameseLib, Success, NeedMoreData, Disabled
    lib = SiameseLib(%(lib)r).init()
    enc, dec, other = lib.Encoder(), lib.Decoder(), lib.Encoder()
    out = {}
    nums = [enc.add(bytes([i %% 251]) * 100) for i in range(20)]
    out["before"] = [dec.add_original(n, bytes([n %% 251]) * 100) for n in nums[:10]]
    # siamese_encode flushes and synchronises: the first sync fails
    out["encode"] = enc.encode_raw()[0]
    # every later call on every instance is Disabled, including a fresh one
    out["after_enc"] = [enc.add_raw(b"x" * 10)[0], enc.encode_raw()[0], enc.get(0)[0],
                        enc.retransmit()[0]]
    out["after_other"] = [other.add_raw(b"y" * 10)[0], other.encode_raw()[0]]
    out["after_dec"] = [dec.add_original(15, b"z" * 100), dec.add_recovery(b"q" * 20),
                        dec.decode_raw()[0], dec.get(0)[0], dec.ack()[0]]
    late = lib.Encoder()
    out["fresh"] = [late.add_raw(b"w" * 10)[0]]
    print(json.dumps(out))
""")


def run_child(fail_at):
    env = dict(os.environ, HOSTSIM_FAIL_SYNC=str(fail_at))
    code = CHILD % {"root": ROOT, "lib": os.path.join(ROOT, "tests", "hostsim",
                                                       "libsiamese_hostsim.so")}
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    import json
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_sync_failure_disables_every_instance():
    from siamese_amd.binding import Success, Disabled
    r = run_child(1)
    assert r["before"] == [Success] * 10
    assert r["encode"] == Disabled
    assert r["after_enc"] == [Disabled] * 4
    assert r["after_other"] == [Disabled] * 2
    assert r["after_dec"] == [Disabled] * 5
    assert r["fresh"] == [Disabled]


def test_no_failure_without_injection():
    from siamese_amd.binding import Success, Disabled
    r = run_child(0)
    assert r["encode"] == Success
    assert Disabled not in r["after_enc"] + r["after_other"] + r["after_dec"] + r["fresh"]


def test_batch_flush_reports_failure():
    """sgpu_submit / sgpu_flush return nonzero once the device failed, and the
    batch driver stops with an error instead of reading stale results."""
    code = textwrap.dedent(r"""
        import sys
        sys.path.insert(0, %(tests)r)
        import scenario_lib as S
        cfg = S.replace(S.CONFIGS["C4"], streams=4)
        try:
            S.run_batch(S.SIM_LIB, cfg, verify=False)
        except RuntimeError as e:
            print("failed:", e)
        else:
            print("completed")
    """) % {"tests": os.path.join(ROOT, "tests")}
    env = dict(os.environ, HOSTSIM_FAIL_SYNC="1")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    assert "failed:" in p.stdout and "rc=-3" in p.stdout, p.stdout
