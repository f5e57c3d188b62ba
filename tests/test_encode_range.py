"""sgpu_encode_range: N recovery packets in one call, bit-exact with N
sgpu_encode calls (reference siamese_encode, siamese.cpp:159-168, per packet;
SiameseEncoder.cpp:1146-1254).  CPU test double of the backend (tests/hostsim),
whose kernels are the reference arithmetic; the GPU suite runs the headline
through it (the block-mode harness encodes in ranges, fixture C4x1024hr).

Two encoders take the same originals; one makes its packets by single calls,
the other by one range call (chunked internally past 64 packets), and every
packet's bytes, length, footer and head must agree, as must every packet of
a range after the call returns (each stays valid until the next encode).
"""
import ctypes as C
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, "tests", "hostsim", "libsiamese_hostsim.so")


class Rec(C.Structure):
    _fields_ = [("DeviceData", C.c_void_p), ("DataBytes", C.c_uint), ("FooterBytes", C.c_uint),
                ("Footer", C.c_ubyte * 8), ("Head", C.c_ubyte * 4), ("Producer", C.c_void_p)]


_L = None


def lib():
    global _L
    if _L is None:
        L = C.CDLL(SIM)
        L.sgpu_encoder_create.restype = C.c_void_p
        L.sgpu_device_alloc.restype = C.c_void_p
        for f in ("sgpu_encoder_add", "sgpu_encode", "sgpu_encode_range", "sgpu_flush", "sgpu_gather"):
            getattr(L, f).restype = C.c_int
        assert L.sgpu_init(-1) == 0
        _L = L
    return _L


def make_encoder(L, dev, sizes, remove_before=None):
    enc = C.c_void_p(L.sgpu_encoder_create())
    for i, b in enumerate(sizes):
        num = C.c_uint(0)
        assert L.sgpu_encoder_add(enc, C.c_void_p(dev + 2048 * i), b, C.byref(num)) == 0
    if remove_before is not None:
        assert L.sgpu_encoder_remove_before(enc, remove_before) == 0
    return enc


def packet_bytes(L, recs):
    assert L.sgpu_flush() == 0
    out = []
    for r in recs:
        buf = (C.c_ubyte * max(1, r.DataBytes))()
        srcs = (C.c_void_p * 1)(r.DeviceData)
        lens = (C.c_uint * 1)(r.DataBytes)
        assert L.sgpu_gather(1, srcs, lens, buf) == 0
        out.append((bytes(buf[:r.DataBytes]), r.DataBytes, r.FooterBytes, bytes(r.Footer[:r.FooterBytes]),
                    bytes(r.Head)))
    return out


@pytest.mark.parametrize("originals,count,var", [(1, 3, False), (7, 5, True), (40, 70, False),
                                                 (300, 130, True), (256, 64, False)])
def test_range_matches_single_calls(originals, count, var):
    L = lib()
    dev = L.sgpu_device_alloc(C.c_size_t(2048 * originals))
    host = bytes((i * 131 + 7) % 251 for i in range(2048 * originals))
    L.sgpu_h2d(C.c_void_p(dev), host, C.c_size_t(len(host)))
    sizes = [(1200 if not var else 40 + (i * 97) % 1300) for i in range(originals)]
    a = make_encoder(L, dev, sizes)
    b = make_encoder(L, dev, sizes)
    singles = []
    for _ in range(count):
        r = Rec()
        assert L.sgpu_encode(a, C.byref(r)) == 0
        singles.append(packet_bytes(L, [r])[0])   # (valid until a's next encode)
    recs = (Rec * count)()
    made = C.c_uint(0)
    assert L.sgpu_encode_range(b, recs, count, C.byref(made)) == 0
    assert made.value == count
    got = packet_bytes(L, list(recs))   # every packet of the range, read after the call
    assert got == singles
    # the next packet after a range is the next single call's
    ra, rb = Rec(), Rec()
    assert L.sgpu_encode(a, C.byref(ra)) == 0
    assert L.sgpu_encode(b, C.byref(rb)) == 0
    assert packet_bytes(L, [ra]) == packet_bytes(L, [rb])
    L.sgpu_encoder_free(a)
    L.sgpu_encoder_free(b)


def test_range_stops_where_a_call_would_fail():
    L = lib()
    enc = C.c_void_p(L.sgpu_encoder_create())
    recs = (Rec * 4)()
    made = C.c_uint(7)
    # nothing added: the first call returns NeedMoreData (siamese_encode's result)
    assert L.sgpu_encode_range(enc, recs, 4, C.byref(made)) == 2
    assert made.value == 0 and recs[0].DataBytes == 0
    assert L.sgpu_encode_range(enc, recs, 0, C.byref(made)) == 0 and made.value == 0
    assert L.sgpu_encode_range(None, recs, 4, C.byref(made)) == 1
    L.sgpu_encoder_free(enc)
