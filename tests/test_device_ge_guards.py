"""sgpu_decode_device's pending matrix job, at the edges (CPU test double of the
backend, tests/hostsim; the GPU suite runs the same calls through the HIP
library in test_gpu_parity.py).

* A flush that fails while a decoder's matrix job is in it delivers no
  completions (Engine::wait), so the job's result never arrives: the decoder
  must report Siamese_Disabled (sticky, siamese.h:147-150) instead of
  SGPU_DECODE_PENDING forever, and its other calls must answer as a disabled
  decoder does, not InvalidInput.
* sgpu_frames_recv must not hand a frame to a decoder whose job is pending
  (the job was built from the decoder's window as it stood): the frame's
  result is InvalidInput, as every other sgpu_decoder_* call returns then.

Each case runs in a child process: a failed engine is process-wide.
"""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, "tests", "hostsim", "libsiamese_hostsim.so")

CHILD = textwrap.dedent(r"""
    import ctypes as C, json, sys
    L = C.CDLL(%(lib)r)
    class Rec(C.Structure):
        _fields_ = [("DeviceData", C.c_void_p), ("DataBytes", C.c_uint), ("FooterBytes", C.c_uint),
                    ("Footer", C.c_ubyte * 8), ("Head", C.c_ubyte * 4), ("Producer", C.c_void_p)]
    class Orig(C.Structure):
        _fields_ = [("PacketNum", C.c_uint), ("Data", C.c_void_p), ("DataBytes", C.c_uint)]
    L.sgpu_encoder_create.restype = C.c_void_p
    L.sgpu_decoder_create.restype = C.c_void_p
    L.sgpu_device_alloc.restype = C.c_void_p
    L.sgpu_host_alloc.restype = C.c_void_p
    for f in ("sgpu_encoder_add", "sgpu_encode", "sgpu_decoder_add_original", "sgpu_decoder_add_recovery",
              "sgpu_decode_device", "sgpu_decoder_is_ready", "sgpu_frames_recv", "sgpu_decoder_get"):
        getattr(L, f).restype = C.c_int
    out = {"init": L.sgpu_init(-1)}
    enc, dec = C.c_void_p(L.sgpu_encoder_create()), C.c_void_p(L.sgpu_decoder_create())
    N, B, LOST = 24, 200, (3, 7, 11)
    dev = L.sgpu_device_alloc(C.c_size_t(N * 256))
    host = bytes((i * 7 + k) %% 251 for i in range(N) for k in range(256))
    L.sgpu_h2d(C.c_void_p(dev), host, C.c_size_t(N * 256))
    for i in range(N):
        num = C.c_uint(0)
        assert L.sgpu_encoder_add(enc, C.c_void_p(dev + 256 * i), B, C.byref(num)) == 0
        if i not in LOST:
            assert L.sgpu_decoder_add_original(dec, num.value, C.c_void_p(dev + 256 * i), B) == 0
    recs = []
    for _ in range(len(LOST)):
        r = Rec()
        assert L.sgpu_encode(enc, C.byref(r)) == 0
        recs.append(r)
        assert L.sgpu_decoder_add_recovery(dec, C.byref(r)) == 0
    out["flush1"] = L.sgpu_flush()
    p, n = C.POINTER(Orig)(), C.c_uint(0)
    out["decode1"] = L.sgpu_decode_device(dec, C.byref(p), C.byref(n))
    if %(frame)d:
        # a received original arriving as a frame while the job is pending
        hb = L.sgpu_frame_header_bytes(0, B)
        fh = (C.c_ubyte * (hb + B))()
        L.sgpu_frame_write_header(0, 0, LOST[0], B, fh)
        fdev = L.sgpu_device_alloc(C.c_size_t(hb + B + 64))
        L.sgpu_h2d(C.c_void_p(fdev), fh, C.c_size_t(hb + B))
        decs = (C.c_void_p * 1)(dec.value)
        res, cnt = (C.c_int * 1)(), C.c_uint(0)
        out["recv"] = L.sgpu_frames_recv(decs, 1, fh, C.c_void_p(fdev), C.c_size_t(hb + B), res, 1, C.byref(cnt))
        out["recv_result"] = res[0]
        out["recv_count"] = cnt.value
    out["flush2"] = L.sgpu_flush()
    out["decode2"] = L.sgpu_decode_device(dec, C.byref(p), C.byref(n))
    out["decode2_count"] = n.value
    out["is_ready"] = L.sgpu_decoder_is_ready(dec)
    out["decode3"] = L.sgpu_decode_device(dec, C.byref(p), C.byref(n))
    if out["decode2"] == 0:
        got = []
        for k in range(N):
            o = Orig()
            o.PacketNum = k
            got.append(L.sgpu_decoder_get(dec, C.byref(o)))
        out["gets"] = got
    print(json.dumps(out))
""")

Success, InvalidInput, NeedMoreData, Disabled, Pending = 0, 1, 2, 5, 6


def run_child(fail_at=0, frame=False):
    env = dict(os.environ, HOSTSIM_FAIL_SYNC=str(fail_at))
    p = subprocess.run([sys.executable, "-c", CHILD % {"lib": SIM, "frame": int(frame)}], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_pending_job_completes_without_failure():
    r = run_child(0)
    assert r["init"] == 0 and r["flush1"] == 0 and r["flush2"] == 0
    assert r["decode1"] == Pending
    assert r["decode2"] == Success and r["decode2_count"] == 3
    assert r["gets"] == [Success] * 24


def test_failed_flush_with_pending_job_disables_the_decoder():
    """the decoder used to return PENDING forever (geDone never set)
    and every other call InvalidInput."""
    # (the third synchronisation: sgpu_h2d's, flush1's, then the flush carrying the job)
    r = run_child(3)
    assert r["flush1"] == 0 and r["decode1"] == Pending
    assert r["flush2"] != 0
    assert r["decode2"] == Disabled
    # not InvalidInput (the job no longer holds the decoder): NeedMoreData, as
    # the reference's IsReadyToDecode answers once EmergencyDisabled
    # (SiameseDecoder.h:565-571, SiameseDecoder.cpp:541-545)
    assert r["is_ready"] == NeedMoreData
    assert r["decode3"] == Disabled


def test_frames_recv_skips_a_decoder_with_a_pending_job():
    """frames_recv called add_original directly, bypassing the
    ge_pending guard; the frame must be refused and the job's decode must
    still recover exactly the packets it was built for."""
    r = run_child(0, frame=True)
    assert r["decode1"] == Pending
    assert r["recv_count"] == 1 and r["recv_result"] == InvalidInput and r["recv"] == InvalidInput
    assert r["decode2"] == Success and r["decode2_count"] == 3
    assert r["gets"] == [Success] * 24
