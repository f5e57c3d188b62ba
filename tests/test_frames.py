"""f2: framed datagrams -- bulk packet ingest and egress of the batch API
(include/siamese_gpu.h, "Framed datagrams"; siamese_amd/csrc/frames.cpp).

A frame is [length prefix (reference SiameseSerializers.h:566-593)][type]
[flow][PacketNum (originals)][data]; recovery packets carry their metadata
footer (SiameseSerializers.h:736-800), which the ingest parses from the host
copy while the bytes are copied from the staged device copy.

* the header writer and the bulk parser round-trip, padding (zero bytes) is
  skipped and malformed input is rejected;
* one sgpu_frames_recv call routes a ring of interleaved frames to many
  decoders (per-frame result codes);
* the loopback workloads with every original arriving as a frame and every
  recovery packet leaving as one (harness frames mode) reproduce the
  reference's golden digests -- on the CPU test double here and on the
  MI355X in the gpu-marked test.
"""
import ctypes
import random

import pytest

import golden
import scenario_lib as S


class Frame(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint) for n in ("Type", "Flow", "PacketNum", "Offset", "Bytes")]


def _lib(path):
    L = ctypes.CDLL(path)
    L.sgpu_frame_header_bytes.restype = ctypes.c_uint
    L.sgpu_frame_header_bytes.argtypes = [ctypes.c_uint, ctypes.c_uint]
    L.sgpu_frame_write_header.restype = ctypes.c_uint
    L.sgpu_frame_write_header.argtypes = [ctypes.c_uint] * 4 + [ctypes.c_void_p]
    L.sgpu_frames_parse.restype = ctypes.c_int
    L.sgpu_frames_parse.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Frame), ctypes.c_uint,
                                    ctypes.POINTER(ctypes.c_uint)]
    return L


def _frame(L, ftype, flow, num, data):
    hdr = ctypes.create_string_buffer(16)
    h = L.sgpu_frame_write_header(ftype, flow, num, len(data), hdr)
    assert h == L.sgpu_frame_header_bytes(ftype, len(data)) > 0
    return hdr.raw[:h] + bytes(data)


def test_frames_round_trip_with_padding():
    L = _lib(S.SIM_LIB)
    rng = random.Random(7)
    want, ring = [], b""
    for _ in range(300):
        ftype = rng.randrange(2)
        flow = rng.randrange(1 << 24)
        num = rng.randrange(1 << 22) if ftype == 0 else 0
        data = bytes(rng.randrange(256) for _ in range(rng.choice([1, 2, 120, 127, 128, 1400, 16400])))
        off = len(ring) + L.sgpu_frame_header_bytes(ftype, len(data))
        ring += _frame(L, ftype, flow, num, data)
        want.append((ftype, flow, num, off, len(data)))
        ring += b"\0" * rng.randrange(4)       # zero bytes between frames: empty frames
    out = (Frame * 400)()
    n = ctypes.c_uint()
    assert L.sgpu_frames_parse(ring, len(ring), out, 400, ctypes.byref(n)) == 0
    got = [(f.Type, f.Flow, f.PacketNum, f.Offset, f.Bytes) for f in out[:n.value]]
    assert got == want
    # the length prefix is the reference's symbol header (SiameseSerializers.h:566-593)
    assert _frame(L, 1, 5, 0, b"x" * 1400)[:2] == bytes([0x85, 0x7c])   # 1404 = 0x57c


def test_frames_parse_rejects_malformed():
    L = _lib(S.SIM_LIB)
    out = (Frame * 8)()
    n = ctypes.c_uint()
    good = _frame(L, 0, 1, 2, b"abc")
    for bad in (good[:-1],                         # truncated
                bytes([4, 7]) + b"abcd",           # unknown type
                bytes([3, 0, 1, 0]),               # original without a PacketNum / payload
                bytes([0x85]),                     # cut-off length prefix
                ):
        assert L.sgpu_frames_parse(bad, len(bad), out, 8, ctypes.byref(n)) != 0
    # more frames than room: not all consumed
    two = good + good
    assert L.sgpu_frames_parse(two, len(two), out, 1, ctypes.byref(n)) != 0 and n.value == 1


def test_bulk_recv_routes_interleaved_frames():
    """One sgpu_frames_recv call hands a ring of interleaved originals of 6
    flows to their decoders: per-frame results (a duplicate reads
    DuplicateData, an unknown flow InvalidInput) and the packets present."""
    L = _lib(S.SIM_LIB)
    assert L.sgpu_init(-1) == 0
    L.sgpu_decoder_create.restype = ctypes.c_void_p
    L.sgpu_decoder_free.argtypes = [ctypes.c_void_p]
    L.sgpu_decoder_has.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    L.sgpu_device_alloc.restype = ctypes.c_void_p
    L.sgpu_device_alloc.argtypes = [ctypes.c_size_t]
    L.sgpu_device_free.argtypes = [ctypes.c_void_p]
    L.sgpu_h2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.sgpu_flush.restype = ctypes.c_int
    L.sgpu_frames_recv.restype = ctypes.c_int
    L.sgpu_frames_recv.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.c_uint,
                                   ctypes.POINTER(ctypes.c_uint)]
    decs = (ctypes.c_void_p * 6)(*[L.sgpu_decoder_create() for _ in range(6)])
    ring, expect = b"", []
    for num in range(5):
        for flow in range(6):
            ring += _frame(L, 0, flow, num, bytes([flow, num]) * 50)
            expect.append(0)
    ring += _frame(L, 0, 2, 3, b"dup" * 10)      # duplicate of flow 2's #3
    expect.append(4)                              # Siamese_DuplicateData
    ring += _frame(L, 0, 9, 0, b"nowhere")       # flow without a decoder
    expect.append(1)                              # Siamese_InvalidInput
    dev = L.sgpu_device_alloc(len(ring))
    host = ctypes.create_string_buffer(ring, len(ring))
    assert L.sgpu_h2d(dev, host, len(ring)) == 0
    res = (ctypes.c_int * 64)()
    n = ctypes.c_uint()
    L.sgpu_frames_recv(decs, 6, host, dev, len(ring), res, 64, ctypes.byref(n))
    assert n.value == len(expect)
    assert list(res[:n.value]) == expect
    assert L.sgpu_flush() == 0
    for flow in range(6):
        for num in range(5):
            assert L.sgpu_decoder_has(decs[flow], num) == 0
        assert L.sgpu_decoder_has(decs[flow], 5) == 2
    for d in decs:
        L.sgpu_decoder_free(d)
    L.sgpu_device_free(dev)


def test_frames_parse_returns_frames_before_malformed():
    """A malformed frame in the middle of a ring: the frames before it are
    returned (with InvalidInput), nothing after it."""
    L = _lib(S.SIM_LIB)
    good = [_frame(L, 0, 1, k, bytes([k]) * 40) for k in range(3)]
    ring = good[0] + good[1] + bytes([4, 7]) + b"abcd" + good[2]
    out = (Frame * 8)()
    n = ctypes.c_uint()
    assert L.sgpu_frames_parse(ring, len(ring), out, 8, ctypes.byref(n)) != 0
    assert n.value == 2 and [f.PacketNum for f in out[:2]] == [0, 1]


def test_bulk_recv_delivers_frames_before_malformed():
    """sgpu_frames_recv over a ring with one corrupt datagram in the middle
    of a 256-frame parse block: every frame before it reaches its decoder and
    is counted; the call reports InvalidInput and reads no further."""
    L = _lib(S.SIM_LIB)
    assert L.sgpu_init(-1) == 0
    L.sgpu_decoder_create.restype = ctypes.c_void_p
    L.sgpu_decoder_free.argtypes = [ctypes.c_void_p]
    L.sgpu_decoder_has.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    L.sgpu_device_alloc.restype = ctypes.c_void_p
    L.sgpu_device_alloc.argtypes = [ctypes.c_size_t]
    L.sgpu_device_free.argtypes = [ctypes.c_void_p]
    L.sgpu_h2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.sgpu_flush.restype = ctypes.c_int
    L.sgpu_frames_recv.restype = ctypes.c_int
    L.sgpu_frames_recv.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.c_uint,
                                   ctypes.POINTER(ctypes.c_uint)]
    decs = (ctypes.c_void_p * 1)(L.sgpu_decoder_create())
    # 300 good frames (past the first 256-frame block), a corrupt one, 5 more
    ring = b"".join(_frame(L, 0, 0, k, bytes([k & 255]) * 20) for k in range(300))
    ring += bytes([0x85])                                    # cut-off length prefix...
    ring += bytes([9, 9, 9])                                 # ...with garbage after it
    ring += b"".join(_frame(L, 0, 0, k, b"late" * 5) for k in range(300, 305))
    dev = L.sgpu_device_alloc(len(ring))
    host = ctypes.create_string_buffer(ring, len(ring))
    assert L.sgpu_h2d(dev, host, len(ring)) == 0
    res = (ctypes.c_int * 400)()
    n = ctypes.c_uint()
    assert L.sgpu_frames_recv(decs, 1, host, dev, len(ring), res, 400, ctypes.byref(n)) == 1   # InvalidInput
    assert n.value == 300 and list(res[:300]) == [0] * 300
    assert L.sgpu_flush() == 0
    assert all(L.sgpu_decoder_has(decs[0], k) == 0 for k in (0, 255, 256, 299))
    assert L.sgpu_decoder_has(decs[0], 300) == 2
    L.sgpu_decoder_free(decs[0])
    L.sgpu_device_free(dev)


def test_frames_send_rejects_empty_and_oversized():
    """sgpu_frames_send frames no packet sgpu_frame_write_header would refuse
    (a 0-byte packet would be a bare header the receiver rejects)."""
    L = _lib(S.SIM_LIB)
    assert L.sgpu_init(-1) == 0

    class Rec(ctypes.Structure):
        _fields_ = [("DeviceData", ctypes.c_void_p), ("DataBytes", ctypes.c_uint), ("FooterBytes", ctypes.c_uint),
                    ("Footer", ctypes.c_ubyte * 8), ("Head", ctypes.c_ubyte * 4), ("Producer", ctypes.c_void_p)]

    L.sgpu_frames_send.restype = ctypes.c_longlong
    L.sgpu_frames_send.argtypes = [ctypes.c_uint, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint), ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    L.sgpu_device_alloc.restype = ctypes.c_void_p
    L.sgpu_device_alloc.argtypes = [ctypes.c_size_t]
    L.sgpu_device_free.argtypes = [ctypes.c_void_p]
    L.sgpu_host_alloc.restype = ctypes.c_void_p
    L.sgpu_host_alloc.argtypes = [ctypes.c_size_t]
    L.sgpu_host_free.argtypes = [ctypes.c_void_p]
    dev = L.sgpu_device_alloc(4096)
    pinned = L.sgpu_host_alloc(1 << 20)
    flows = (ctypes.c_uint * 1)(3)
    used = ctypes.c_size_t()
    for bad in (0, 536870912):   # (SIAMESE_MAX_PACKET_BYTES + 1)
        pk = Rec(dev, bad)
        assert L.sgpu_frames_send(1, ctypes.byref(pk), flows, pinned, 1 << 20, ctypes.byref(used)) == -1
    L.sgpu_host_free(pinned)
    L.sgpu_device_free(dev)


@pytest.mark.parametrize("name", ["C1", "C1var", "C2x64", "smoke_C4x8", "edge_var_block", "edge_lag"])
def test_hostsim_frames_match_golden(name):
    """Originals arrive as frames in a pinned ring (staged per job) and go
    through sgpu_frames_recv; recovery packets leave as frames
    (sgpu_frames_send) and their bytes are hashed from the parsed landing:
    the reference's digests, two pipelined steps."""
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, e2e=True, frames=True, steps=2, threads=4,
                           groups=2 if cfg.streams >= 8 else 1)
    assert rep.mismatches == 0 and rep.checked > 0
    assert S.digests(res) == golden.load(name)["digests"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C1", "C1var", "C2x64", "C4x256", "edge_var_block"])
@pytest.mark.parametrize("defer", [0, 4])
def test_gpu_frames_match_golden(name, defer):
    cfg = golden.config(name)
    res, rep = S.run_batch(S.AMD_LIB, cfg, verify=True, e2e=True, frames=True, steps=2, threads=16,
                           groups=2 if cfg.streams >= 8 else 1, defer=defer)
    assert rep.mismatches == 0 and rep.checked > 0
    assert S.digests(res) == golden.load(name)["digests"]


class RecoveryPacket(ctypes.Structure):
    _fields_ = [("DeviceData", ctypes.c_void_p), ("DataBytes", ctypes.c_uint), ("FooterBytes", ctypes.c_uint),
                ("Footer", ctypes.c_ubyte * 8), ("Head", ctypes.c_ubyte * 4), ("Producer", ctypes.c_void_p)]


class OriginalPacket(ctypes.Structure):
    _fields_ = [("PacketNum", ctypes.c_uint), ("DataBytes", ctypes.c_uint), ("Data", ctypes.c_void_p)]


def _loopback_over_frames(path):
    """Encoder -> recovery packets framed for egress (sgpu_frames_send) ->
    the landed frame stream, with the originals of a lossy channel, handed to
    a decoder by sgpu_frames_recv (the recovery bytes ingested from the
    staged device copy) -> decode recovers the lost originals byte-exact."""
    L = _lib(path)
    assert L.sgpu_init(0 if "amd" in path else -1) == 0
    for fn in ("sgpu_encoder_create", "sgpu_decoder_create", "sgpu_device_alloc", "sgpu_host_alloc"):
        getattr(L, fn).restype = ctypes.c_void_p
    L.sgpu_device_alloc.argtypes = [ctypes.c_size_t]
    L.sgpu_host_alloc.argtypes = [ctypes.c_size_t]
    for fn in ("sgpu_encoder_free", "sgpu_decoder_free", "sgpu_device_free", "sgpu_host_free"):
        getattr(L, fn).argtypes = [ctypes.c_void_p]
    L.sgpu_h2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.sgpu_h2d_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.sgpu_encoder_add.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.POINTER(ctypes.c_uint)]
    L.sgpu_encode.argtypes = [ctypes.c_void_p, ctypes.POINTER(RecoveryPacket)]
    L.sgpu_frames_send.restype = ctypes.c_longlong
    L.sgpu_frames_send.argtypes = [ctypes.c_uint, ctypes.POINTER(RecoveryPacket), ctypes.POINTER(ctypes.c_uint),
                                   ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    L.sgpu_gather_wait.argtypes = [ctypes.c_longlong]
    L.sgpu_frames_recv.restype = ctypes.c_int
    L.sgpu_frames_recv.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.c_uint,
                                   ctypes.POINTER(ctypes.c_uint)]
    L.sgpu_decoder_is_ready.argtypes = [ctypes.c_void_p]
    L.sgpu_decode.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.POINTER(OriginalPacket)),
                              ctypes.POINTER(ctypes.c_uint)]
    L.sgpu_gather.argtypes = [ctypes.c_uint, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint),
                              ctypes.c_void_p]
    rng = random.Random(3)
    N, size = 40, 1000
    payloads = [bytes(rng.randrange(256) for _ in range(size)) for _ in range(N)]
    lost = {3, 17, 30}
    enc = L.sgpu_encoder_create()
    src = L.sgpu_device_alloc(N * size)
    buf = ctypes.create_string_buffer(b"".join(payloads), N * size)
    assert L.sgpu_h2d(src, buf, N * size) == 0
    num = ctypes.c_uint()
    for i in range(N):
        assert L.sgpu_encoder_add(enc, src + i * size, size, ctypes.byref(num)) == 0 and num.value == i
    recs = (RecoveryPacket * 6)()
    for k in range(6):
        assert L.sgpu_encode(enc, ctypes.byref(recs[k])) == 0
    assert L.sgpu_flush() == 0
    # egress: the recovery packets as frames (flow 0) in pinned memory
    cap = 6 * (size + 64)
    egress = L.sgpu_host_alloc(cap)
    flows = (ctypes.c_uint * 6)()
    used = ctypes.c_size_t()
    t = L.sgpu_frames_send(6, recs, flows, egress, cap, ctypes.byref(used))
    assert t > 0 and L.sgpu_gather_wait(t) == 0
    out = (Frame * 8)()
    n = ctypes.c_uint()
    assert L.sgpu_frames_parse(egress, used.value, out, 8, ctypes.byref(n)) == 0 and n.value == 6
    assert all(f.Type == 1 and f.Bytes == recs[k].DataBytes for k, f in enumerate(out[:6]))
    # ingress: the surviving originals, then the recovery frames, in one ring
    ring = b"".join(_frame(L, 0, 0, i, payloads[i]) for i in range(N) if i not in lost)
    ring += ctypes.string_at(egress, used.value)
    host = L.sgpu_host_alloc(len(ring))
    ctypes.memmove(host, ring, len(ring))
    dev = L.sgpu_device_alloc(len(ring))
    assert L.sgpu_h2d_async(dev, host, len(ring)) == 0
    dec = L.sgpu_decoder_create()
    decs = (ctypes.c_void_p * 1)(dec)
    res = (ctypes.c_int * 64)()
    assert L.sgpu_frames_recv(decs, 1, host, dev, len(ring), res, 64, ctypes.byref(n)) == 0
    assert n.value == N - len(lost) + 6 and not any(res[:n.value])
    assert L.sgpu_decoder_is_ready(dec) == 0
    pk = ctypes.POINTER(OriginalPacket)()
    cnt = ctypes.c_uint()
    assert L.sgpu_decode(dec, ctypes.byref(pk), ctypes.byref(cnt)) == 0
    assert L.sgpu_flush() == 0
    got = sorted(pk[i].PacketNum for i in range(cnt.value))
    assert got == sorted(lost)
    srcs = (ctypes.c_void_p * 3)(*[pk[i].Data for i in range(cnt.value)])
    lens = (ctypes.c_uint * 3)(*[pk[i].DataBytes for i in range(cnt.value)])
    back = ctypes.create_string_buffer(3 * size)
    assert L.sgpu_gather(3, srcs, lens, back) == 0
    for i in range(cnt.value):
        assert back.raw[i * size:(i + 1) * size] == payloads[pk[i].PacketNum]
    L.sgpu_decoder_free(dec)
    L.sgpu_encoder_free(enc)
    for p in (src, dev):
        L.sgpu_device_free(p)
    for p in (egress, host):
        L.sgpu_host_free(p)


def test_hostsim_recovery_frames_loopback():
    _loopback_over_frames(S.SIM_LIB)


@pytest.mark.gpu
def test_gpu_recovery_frames_loopback():
    _loopback_over_frames(S.AMD_LIB)
