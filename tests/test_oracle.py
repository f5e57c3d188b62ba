"""Pin the C oracle restatement (oracle/gf256_oracle.c) to the reference's own
known answers: its GF(256) self-test (gf256.cpp:84-189), its serializer tests
(tests/test_serializers.cpp) and known answers produced by the compiled
reference.  CPU only."""
import ctypes
import os
import struct

import pytest

import scenario_lib as S

ORACLE = os.path.join(S.ROOT, "oracle", "_ref", "libgf256_oracle.so")


@pytest.fixture(scope="module")
def orc():
    L = ctypes.CDLL(ORACLE)
    u8 = ctypes.c_uint8
    for name, res, args in [
        ("orc_init", ctypes.c_int, []),
        ("orc_mul", u8, [u8, u8]), ("orc_div", u8, [u8, u8]), ("orc_inv", u8, [u8]),
        ("orc_sqr", u8, [u8]), ("orc_exp", u8, [ctypes.c_uint]), ("orc_log", ctypes.c_uint, [u8]),
        ("orc_poly", ctypes.c_uint, []),
        ("orc_column_value", u8, [ctypes.c_uint]), ("orc_row_value", u8, [ctypes.c_uint]),
        ("orc_row_opcode", ctypes.c_uint, [ctypes.c_uint, ctypes.c_uint]),
        ("orc_cauchy_element", u8, [ctypes.c_uint, ctypes.c_uint]),
        ("orc_write_footer", ctypes.c_uint, [ctypes.c_uint] * 4 + [ctypes.c_char_p]),
        ("orc_write_length", ctypes.c_uint, [ctypes.c_uint, ctypes.c_char_p]),
    ]:
        getattr(L, name).restype = res
        getattr(L, name).argtypes = args
    assert L.orc_init() == 0
    return L


def test_field_tables(orc):
    assert orc.orc_poly() == 0x14D
    assert [orc.orc_exp(i) for i in range(10)] == [1, 2, 4, 8, 0x10, 0x20, 0x40, 0x80, 0x4d, 0x9a]
    assert [orc.orc_log(i) for i in range(1, 10)] == [255, 1, 23, 2, 46, 24, 83, 3, 106]
    assert orc.orc_mul(2, 0x80) == 0x4d
    assert orc.orc_mul(0x53, 0xca) == 0x94
    assert orc.orc_inv(2) == 0xa6
    assert orc.orc_sqr(3) == 0x05
    assert orc.orc_div(1, 3) == 0xc4


def test_reference_self_test_vectors(orc):
    # gf256.cpp:96-117: exhaustive mul/div consistency
    for i in range(256):
        for j in range(256):
            p = orc.orc_mul(i, j)
            if i and j:
                assert orc.orc_div(p, i) == j and orc.orc_div(p, j) == i
            else:
                assert p == 0
            if j == 1:
                assert p == i
    # gf256.cpp:119-186: bulk-op vectors on a 63-byte buffer with canaries
    n = 63
    A = (ctypes.c_uint8 * (n + 1))(*([0x1f] * n + [0x5a]))
    B = (ctypes.c_uint8 * (n + 1))(*([0xf7] * n + [0x5a]))
    orc.orc_add_mem(A, B, n)
    assert list(A[:n]) == [0x1f ^ 0xf7] * n and A[n] == 0x5a
    A = (ctypes.c_uint8 * (n + 1))(*([0xff] * n + [0x5a]))
    B = (ctypes.c_uint8 * (n + 1))(*([0xaa] * n + [0x5a]))
    orc.orc_muladd_mem(A, ctypes.c_uint8(0x6c), B, n)
    assert list(A[:n]) == [orc.orc_mul(0xaa, 0x6c) ^ 0xff] * n and A[n] == 0x5a
    A = (ctypes.c_uint8 * (n + 1))(*([0xff] * n + [0x5a]))
    B = (ctypes.c_uint8 * (n + 1))(*([0x55] * n + [0x5a]))
    orc.orc_mul_mem(A, B, ctypes.c_uint8(0xa2), n)
    assert list(A[:n]) == [orc.orc_mul(0xa2, 0x55)] * n and A[n] == 0x5a


def test_code_definition(orc):
    assert [orc.orc_column_value(c) for c in range(10)] == [3, 202, 148, 94, 40, 239, 185, 131, 77, 23]
    assert [orc.orc_row_value(r) for r in range(10)] == list(range(2, 12))
    assert [orc.orc_row_opcode(l, 0) for l in range(8)] == [23, 54, 36, 54, 56, 48, 41, 2]
    assert [orc.orc_row_opcode(l, 1) for l in range(8)] == [1, 1, 20, 6, 1, 14, 50, 26]
    assert [orc.orc_cauchy_element(0, c) for c in range(8)] == [0x6b, 0x29, 0xe9, 0xa4, 0xff, 0x69,
                                                               0xe7, 0x5a]
    # opcode 0 is remapped to 16 (SiameseCommon.h:173)
    assert all(orc.orc_row_opcode(l, r) != 0 for l in range(8) for r in range(255))


def test_pcg(orc):
    out = (ctypes.c_uint32 * 4)()
    orc.orc_pcg(ctypes.c_uint64(0), ctypes.c_uint64(1), out, 4)
    assert list(out) == [0xe2393051, 0x01112f35, 0xd3509d35, 0x0b932f4a]
    orc.orc_pcg(ctypes.c_uint64(1013), ctypes.c_uint64(0), out, 4)
    assert list(out) == [0xbbc743b4, 0x7086af75, 0x7130138c, 0xcef6c1c8]


def test_footer_known_answer(orc):
    buf = ctypes.create_string_buffer(16)
    n = orc.orc_write_footer(5, 1000, 300, 200, buf)
    assert buf.raw[:n] == bytes.fromhex("05c880e8832b81")


def test_footer_roundtrip_grid(orc):
    # shape of reference tests/test_serializers.cpp:449-526
    buf = ctypes.create_string_buffer(16)
    row, cs, sc, lc = (ctypes.c_uint() for _ in range(4))
    for start in [0, 1, 0x7f, 0x80, 0x3fff, 0x4000, 0x1fffff, 0x3fffff]:
        for s in [1, 2, 127, 128, 129, 16000]:
            for ldpc in sorted({1, s // 2 or 1, s}):
                for r in ([0] if s == 1 else [0, 1, 254]):
                    n = orc.orc_write_footer(r, start, s, ldpc, buf)
                    assert 2 <= n <= 8
                    got = orc.orc_read_footer(buf, n, ctypes.byref(row), ctypes.byref(cs),
                                              ctypes.byref(sc), ctypes.byref(lc))
                    assert got == n
                    assert (cs.value, sc.value) == (start, s)
                    if s > 1:
                        assert (row.value, lc.value) == (r, ldpc)


def test_length_prefix_roundtrip(orc):
    buf = ctypes.create_string_buffer(8)
    out = ctypes.c_uint()
    for v, want in [(1, 1), (0x7f, 1), (0x80, 2), (1400, 2), (0x3fff, 2), (0x4000, 3),
                    (65536, 3), (0x1fffff, 3), (0x200000, 4), (0x1fffffff, 4)]:
        n = orc.orc_write_length(v, buf)
        assert n == want
        assert orc.orc_read_length(buf, n, ctypes.byref(out)) == n and out.value == v
    assert orc.orc_write_length(1400, buf) == 2 and buf.raw[:2] == bytes.fromhex("8578")
    assert orc.orc_write_length(65536, buf) == 3 and buf.raw[:3] == bytes.fromhex("c10000")


def test_nack_roundtrip(orc):
    buf = ctypes.create_string_buffer(16)
    rs, lm = ctypes.c_uint(), ctypes.c_uint()
    for r in [0, 1, 31, 32, 4095, 4096, 0x7ffff, 0x80000, 0x3fffff]:
        for m in [0, 1, 2, 3, 130, 16384 + 5]:
            n = orc.orc_write_nack(r, m, buf)
            assert n <= 7
            assert orc.orc_read_nack(buf, 16, ctypes.byref(rs), ctypes.byref(lm)) == n
            assert (rs.value, lm.value) == (r, m)


def _set_packet(pid, nbytes):
    """reference tests/unit_test.cpp:90-116"""
    out = bytearray()
    st, inc = 0, ((pid << 1) | 1) & (2 ** 64 - 1)

    def nxt():
        nonlocal st
        old = st
        st = (old * 6364136223846793005 + inc) & (2 ** 64 - 1)
        xs = (((old >> 18) ^ old) >> 27) & 0xffffffff
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xffffffff

    nxt()
    st = (st + nbytes) & (2 ** 64 - 1)
    nxt()
    n = nbytes
    if n >= 4:
        out += struct.pack("<I", nbytes)
        n -= 4
    while n >= 4:
        out += struct.pack("<I", nxt())
        n -= 4
    if n:
        x = nxt()
        out += bytes((x >> (8 * k)) & 0xff for k in range(n))
    return bytes(out)


def test_siamese_row_restatement_matches_reference_kat(orc):
    """orc_siamese_row (encoder sums + row mix + LDPC + RX*product) reproduces the
    reference's first Siamese row for 100 SetPacket(i, 16) originals."""
    count = 100
    syms = [bytes([16]) + _set_packet(i, 16) for i in range(count)]
    arrs = [(ctypes.c_uint8 * len(s)).from_buffer_copy(s) for s in syms]
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * count)(*[ctypes.cast(a, ctypes.POINTER(ctypes.c_uint8))
                                                     for a in arrs])
    lens = (ctypes.c_uint * count)(*[len(s) for s in syms])
    out = (ctypes.c_uint8 * 64)()
    orc.orc_siamese_row(ptrs, lens, count, 0, out)
    row = bytes(out[:17])
    foot = ctypes.create_string_buffer(16)
    n = orc.orc_write_footer(0, 0, count, count, foot)
    assert (row + foot.raw[:n]).hex() == "08080000001f4e11352a109de6ffe5f61300640063"
