"""ctypes binding of the siamese.h C ABI, for any library exporting it.

Used with siamese_amd/libsiamese_amd.so (the product), and in tests with the
upstream reference (oracle/_ref/libsiamese_ref.so) and the CPU test double
(tests/hostsim/libsiamese_hostsim.so), so API-level behaviour can be compared
call by call.
"""
import ctypes

SIAMESE_VERSION = 5
Success, InvalidInput, NeedMoreData, MaxPacketsReached, DuplicateData, Disabled = range(6)
RESULT_NAMES = ["Success", "InvalidInput", "NeedMoreData", "MaxPacketsReached",
                "DuplicateData", "Disabled"]


class OriginalPacket(ctypes.Structure):
    _fields_ = [("PacketNum", ctypes.c_uint), ("DataBytes", ctypes.c_uint),
                ("Data", ctypes.POINTER(ctypes.c_ubyte))]


class RecoveryPacket(ctypes.Structure):
    _fields_ = [("DataBytes", ctypes.c_uint), ("Data", ctypes.POINTER(ctypes.c_ubyte))]


class SiameseError(RuntimeError):
    def __init__(self, what, code):
        name = RESULT_NAMES[code] if 0 <= code < 6 else str(code)
        super().__init__("%s -> %s" % (what, name))
        self.code = code


def _bytes(ptr, n):
    return ctypes.string_at(ptr, n) if n else b""


def _buf(data):
    return (ctypes.c_ubyte * max(1, len(data))).from_buffer_copy(data if data else b"\0")


class SiameseLib:
    """All 20 siamese.h entry points of one shared library."""

    def __init__(self, path):
        self.path = path
        L = self.L = ctypes.CDLL(path)
        vp, u, i = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
        P = ctypes.POINTER

        def sig(name, res, args):
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
            return f

        self.init_ = sig("siamese_init_", i, [i])
        self.encoder_create = sig("siamese_encoder_create", vp, [])
        self.encoder_free = sig("siamese_encoder_free", None, [vp])
        self.encoder_is_ready = sig("siamese_encoder_is_ready", i, [vp])
        self.encoder_add = sig("siamese_encoder_add", i, [vp, P(OriginalPacket)])
        self.encoder_get = sig("siamese_encoder_get", i, [vp, P(OriginalPacket)])
        self.encoder_remove_before = sig("siamese_encoder_remove_before", i, [vp, u])
        self.encoder_ack = sig("siamese_encoder_ack", i, [vp, vp, u, P(u)])
        self.encoder_retransmit = sig("siamese_encoder_retransmit", i, [vp, P(OriginalPacket)])
        self.encode = sig("siamese_encode", i, [vp, P(RecoveryPacket)])
        self.encoder_stats = sig("siamese_encoder_stats", i, [vp, P(ctypes.c_uint64), u])
        self.decoder_create = sig("siamese_decoder_create", vp, [])
        self.decoder_free = sig("siamese_decoder_free", None, [vp])
        self.decoder_add_original = sig("siamese_decoder_add_original", i,
                                        [vp, P(OriginalPacket)])
        self.decoder_add_recovery = sig("siamese_decoder_add_recovery", i,
                                        [vp, P(RecoveryPacket)])
        self.decoder_get = sig("siamese_decoder_get", i, [vp, P(OriginalPacket)])
        self.decoder_is_ready = sig("siamese_decoder_is_ready", i, [vp])
        self.decode = sig("siamese_decode", i, [vp, P(P(OriginalPacket)), P(u)])
        self.decoder_ack = sig("siamese_decoder_ack", i, [vp, vp, u, P(u)])
        self.decoder_stats = sig("siamese_decoder_stats", i, [vp, P(ctypes.c_uint64), u])
        self.ready = False

    def init(self):
        if not self.ready:
            rc = self.init_(SIAMESE_VERSION)
            if rc != Success:
                raise RuntimeError("%s: siamese_init failed (%s); an MI355X (gfx950) is "
                                   "required" % (self.path, RESULT_NAMES[rc] if rc < 6 else rc))
            self.ready = True
        return self

    def Encoder(self):
        return Encoder(self)

    def Decoder(self):
        return Decoder(self)


class Encoder:
    def __init__(self, lib):
        self.lib = lib.init()
        self.h = lib.encoder_create()
        if not self.h:
            raise MemoryError("siamese_encoder_create failed")

    def close(self):
        if self.h:
            self.lib.encoder_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def is_ready(self):
        return self.lib.encoder_is_ready(self.h)

    def add_raw(self, data):
        buf = _buf(data)
        p = OriginalPacket(0, len(data), buf)
        rc = self.lib.encoder_add(self.h, ctypes.byref(p))
        return rc, p.PacketNum

    def add(self, data):
        rc, num = self.add_raw(data)
        if rc:
            raise SiameseError("siamese_encoder_add", rc)
        return num

    def encode_raw(self):
        r = RecoveryPacket()
        rc = self.lib.encode(self.h, ctypes.byref(r))
        return rc, (_bytes(r.Data, r.DataBytes) if rc == Success else None)

    def encode(self):
        rc, data = self.encode_raw()
        if rc == NeedMoreData:
            return None
        if rc:
            raise SiameseError("siamese_encode", rc)
        return data

    def remove_before(self, num):
        return self.lib.encoder_remove_before(self.h, num)

    def get(self, num):
        p = OriginalPacket(num, 0, None)
        rc = self.lib.encoder_get(self.h, ctypes.byref(p))
        return rc, (_bytes(p.Data, p.DataBytes) if rc == Success else None)

    def ack(self, message):
        nxt = ctypes.c_uint()
        buf = _buf(message)
        rc = self.lib.encoder_ack(self.h, ctypes.cast(buf, ctypes.c_void_p), len(message),
                                  ctypes.byref(nxt))
        return rc, nxt.value

    def retransmit(self):
        p = OriginalPacket()
        rc = self.lib.encoder_retransmit(self.h, ctypes.byref(p))
        return rc, ((p.PacketNum, _bytes(p.Data, p.DataBytes)) if rc == Success else None)

    def stats(self):
        out = (ctypes.c_uint64 * 9)()
        self.lib.encoder_stats(self.h, out, 9)
        return list(out)


class Decoder:
    def __init__(self, lib):
        self.lib = lib.init()
        self.h = lib.decoder_create()
        if not self.h:
            raise MemoryError("siamese_decoder_create failed")

    def close(self):
        if self.h:
            self.lib.decoder_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def add_original(self, num, data):
        buf = _buf(data)
        p = OriginalPacket(num, len(data), buf)
        return self.lib.decoder_add_original(self.h, ctypes.byref(p))

    def add_recovery(self, data):
        buf = _buf(data)
        r = RecoveryPacket(len(data), buf)
        return self.lib.decoder_add_recovery(self.h, ctypes.byref(r))

    def is_ready(self):
        return self.lib.decoder_is_ready(self.h)

    def decode_raw(self):
        pkts = ctypes.POINTER(OriginalPacket)()
        n = ctypes.c_uint()
        rc = self.lib.decode(self.h, ctypes.byref(pkts), ctypes.byref(n))
        out = None
        if rc == Success:
            out = [(pkts[k].PacketNum, _bytes(pkts[k].Data, pkts[k].DataBytes))
                   for k in range(n.value)]
        return rc, out

    def decode(self):
        rc, out = self.decode_raw()
        if rc == NeedMoreData:
            return None
        if rc:
            raise SiameseError("siamese_decode", rc)
        return out

    def get(self, num):
        p = OriginalPacket(num, 0, None)
        rc = self.lib.decoder_get(self.h, ctypes.byref(p))
        return rc, (_bytes(p.Data, p.DataBytes) if rc == Success else None)

    def ack(self, limit=1024):
        buf = ctypes.create_string_buffer(limit)
        used = ctypes.c_uint()
        rc = self.lib.decoder_ack(self.h, buf, limit, ctypes.byref(used))
        return rc, (buf.raw[:used.value] if rc == Success else None)

    def stats(self):
        out = (ctypes.c_uint64 * 11)()
        self.lib.decoder_stats(self.h, out, 11)
        return list(out)
