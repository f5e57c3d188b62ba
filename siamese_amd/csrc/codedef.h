// codedef.h -- the code definition shared by encoder and decoder control
// planes: matrix coefficient generators, packet-number arithmetic and the two
// wire formats (symbol length prefix, recovery footer).  Every constant and
// formula here is fixed by the reference's bit stream; citations point at
// the definition each one reproduces.
#pragma once

#include "gf.h"
#include <cstdint>

namespace sgpu {

// ---- Code parameters (reference SiameseCommon.h:79-202) -------------------
constexpr unsigned kMaxLossRecovery   = 255;    // :80
constexpr unsigned kColumnValuePeriod = 253;    // :83
constexpr unsigned kRowValuePeriod    = 255;    // :86
constexpr unsigned kColumnPeriod      = 0x400000; // :103 (22-bit packet numbers)
constexpr unsigned kLanes             = 8;      // :131
constexpr unsigned kSums              = 3;      // :138
constexpr unsigned kPairRate          = 16;     // :141
constexpr unsigned kSubwindow         = 64;     // :146
constexpr unsigned kCauchyThreshold   = 64;     // :194
constexpr unsigned kSumResetThreshold = 32;     // :199
constexpr unsigned kCauchyMaxColumns  = 64;     // :201
constexpr unsigned kCauchyMaxRows     = 256 - kCauchyMaxColumns; // :202
constexpr unsigned kRemoveThreshold   = 2 * kSubwindow; // SiameseEncoder.h:334, SiameseDecoder.h:549
constexpr unsigned kMaxPacketsInFlight = 16000; // siamese.h:163
constexpr unsigned kMaxFooterBytes    = 8;      // SiameseSerializers.h:731
constexpr unsigned kMaxLengthPrefix   = 4;      // SiameseSerializers.h:558
constexpr unsigned kAlignBytes        = 32;     // PacketAllocator.h:88 (AVX2 build)

inline unsigned align_up(unsigned v) { return (v + kAlignBytes - 1) & ~(kAlignBytes - 1); }

// Column value CX(c): LCG over 3..255 (SiameseCommon.h:89-93)
inline uint8_t column_value(unsigned column)
{
    return (uint8_t)(3 + (column * 199u) % kColumnValuePeriod);
}

// Row value RX(r) over 1..255 (SiameseCommon.h:95-98)
inline uint8_t row_value(unsigned row)
{
    return (uint8_t)(1 + (row + 1) % kRowValuePeriod);
}

// Packet-number (column) arithmetic modulo 2^22 (SiameseCommon.h:106-127)
inline bool column_delta_negative(unsigned delta) { return delta >= kColumnPeriod / 2; }
inline unsigned column_sub(unsigned a, unsigned b) { return (a - b) % kColumnPeriod; }
inline unsigned column_add(unsigned a, unsigned b) { return (a + b) % kColumnPeriod; }

// Thomas Wang 32-bit integer hash (SiameseCommon.h:150-159)
inline uint32_t wang_hash32(uint32_t k)
{
    k += ~(k << 15);
    k ^= k >> 10;
    k += k << 3;
    k ^= k >> 6;
    k += ~(k << 11);
    k ^= k >> 16;
    return k;
}

// 6-bit opcode selecting which running sums feed a lane of a Siamese row
// (SiameseCommon.h:162-174): bits 0..2 -> recovery, bits 3..5 -> product.
inline unsigned row_opcode(unsigned lane, unsigned row)
{
    const uint32_t op = wang_hash32(lane + (row + 3) * kLanes) & 63u;
    return op ? op : 16u;
}

/// The opcodes of one Siamese row, precomputed for every row number: the
/// sums they select as masks of bit lane*3 + s (mask[0] feeds the recovery
/// row from opcode bits 0..2, mask[1] the product from bits 3..5;
/// SiameseEncoder.cpp:1046-1098) and the raw 3-bit halves per lane (the
/// decoder's matrix rows, SiameseDecoder.cpp:2180-2260).
struct RowSelect
{
    uint32_t mask[2];
    uint8_t opLo[kLanes], opHi[kLanes];
};
/// row < 256 (Siamese rows use 0..254; a footer can carry any byte)
const RowSelect& row_select(unsigned row);

// Cauchy element 1/(X_r ^ Y_c), X_r = r + 64, Y_c = c (SiameseCommon.h:212-218)
inline uint8_t cauchy_element(unsigned row, unsigned column)
{
    return gf_inv((uint8_t)((row + kCauchyMaxColumns) ^ column));
}

// PCG-XSH-RR used to pick the sparse ("LDPC") columns (SiameseTools.h:80-102)
struct Pcg32
{
    uint64_t state = 0, inc = 0;
    void seed(uint64_t y, uint64_t x)
    {
        state = 0;
        inc = (y << 1) | 1u;
        next();
        state += x;
        next();
    }
    uint32_t next()
    {
        const uint64_t s = state;
        state = s * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((s >> 18) ^ s) >> 27);
        const uint32_t r = (uint32_t)(s >> 59);
        return (xs >> r) | (xs << ((32u - r) & 31u));
    }
};

/// a % d for a fixed divisor without a division instruction (Lemire,
/// Kaser & Kurz, "Faster remainder by direct computation", 2019): exact for
/// every 32-bit a and d >= 1.  The LDPC picks take two remainders per pair.
struct FastMod
{
    uint64_t m;
    uint32_t d;
    explicit FastMod(uint32_t divisor) : m(~0ULL / divisor + 1), d(divisor) {}
    uint32_t operator()(uint32_t a) const
    {
        const uint64_t low = m * a;
        return (uint32_t)(((unsigned __int128)low * d) >> 64);
    }
};

/// The LDPC pair picks of Siamese row `row` over a window of n columns
/// (reference SiameseEncoder.cpp:1100-1144, SiameseDecoder.cpp:996-1051 and
/// :2306-2339): PCG.Seed(row, n), then ceil(n/16) pairs of Next() % n, as
/// 2*ceil(n/16) offsets in PCG order (even = row term, odd = product term).
/// The same (row, n) recurs across rows of every stream and on both sides
/// of the channel, so each host thread caches the sequences it computes.
/// The pointer stays valid until the calling thread's next ldpc_offsets().
const uint32_t* ldpc_offsets(unsigned row, unsigned n, unsigned* count);


// ---- Metadata carried in every recovery footer (SiameseCommon.h:364-389) --
struct RowMeta
{
    unsigned row = 0;          // 0..254 (Siamese), 0 parity, 1..192 Cauchy
    unsigned columnStart = 0;  // first summed column
    unsigned sumCount = 0;     // columns in the running sum
    unsigned ldpcCount = 0;    // columns in the sparse/Cauchy range (right-aligned)
};

// ---- Symbol length prefix (SiameseSerializers.h:566-627) ------------------
inline unsigned write_length_prefix(unsigned length, uint8_t* out)
{
    if (length < 0x80) {
        out[0] = (uint8_t)length;
        return 1;
    }
    if (length < 0x4000) {
        out[0] = (uint8_t)(0x80 | (length >> 8));
        out[1] = (uint8_t)length;
        return 2;
    }
    if (length < 0x200000) {
        out[0] = (uint8_t)(0xC0 | (length >> 16));
        out[1] = (uint8_t)(length >> 8);
        out[2] = (uint8_t)length;
        return 3;
    }
    out[0] = (uint8_t)(0xE0 | (length >> 24));
    out[1] = (uint8_t)(length >> 16);
    out[2] = (uint8_t)(length >> 8);
    out[3] = (uint8_t)length;
    return 4;
}

/// Returns prefix bytes (1..4) or -1 if `avail` bytes cannot hold it.
inline int read_length_prefix(const uint8_t* in, unsigned avail, unsigned* length)
{
    if (avail < 1)
        return -1;
    const unsigned top = in[0] >> 6;
    if (top <= 1) {
        *length = in[0];
        return 1;
    }
    if (top == 2) {
        if (avail < 2)
            return -1;
        *length = (((unsigned)in[0] << 8) | in[1]) & 0x3fff;
        return 2;
    }
    if ((in[0] & 0xE0) == 0xC0) {
        if (avail < 3)
            return -1;
        *length = (((unsigned)in[0] << 16) | ((unsigned)in[1] << 8) | in[2]) & 0x1fffff;
        return 3;
    }
    if (avail < 4)
        return -1;
    *length = (((unsigned)in[0] << 24) | ((unsigned)in[1] << 16) | ((unsigned)in[2] << 8) | in[3]) &
              0x1fffffff;
    return 4;
}

// ---- Recovery footer, serialized back-to-front --------------------------
// Layout (SiameseSerializers.h:383-551, 736-800):
//   [Row u8][LDPCCount 1-2B][ColumnStart 1-3B][SumCount-1 1-2B]
// Row and LDPCCount are present only when SumCount > 1.

inline unsigned put_count_tail(unsigned count, uint8_t* out) // :510-526
{
    if (count < 0x80) {
        out[0] = (uint8_t)count;
        return 1;
    }
    out[0] = (uint8_t)count;
    out[1] = (uint8_t)(0x80 | (count >> 8));
    return 2;
}

inline unsigned put_column_tail(unsigned column, uint8_t* out) // :381-400
{
    if (column < 0x80) {
        out[0] = (uint8_t)column;
        return 1;
    }
    if (column < 0x4000) {
        out[0] = (uint8_t)column;
        out[1] = (uint8_t)(0x80 | (column >> 8));
        return 2;
    }
    out[0] = (uint8_t)column;
    out[1] = (uint8_t)(column >> 8);
    out[2] = (uint8_t)(0xC0 | (column >> 16));
    return 3;
}

inline unsigned write_footer(const RowMeta& m, uint8_t* out) // :736-754
{
    unsigned n = 0;
    if (m.sumCount > 1) {
        out[n++] = (uint8_t)m.row;
        n += put_count_tail(m.ldpcCount, out + n);
    }
    n += put_column_tail(m.columnStart, out + n);
    n += put_count_tail(m.sumCount - 1, out + n);
    return n;
}

/// `end` points one past the last byte; `avail` bytes precede it.
inline int get_count_tail(const uint8_t* end, unsigned avail, unsigned* count) // :531-551
{
    if (avail < 1)
        return -1;
    const uint8_t last = end[-1];
    if (!(last & 0x80)) {
        *count = last;
        return 1;
    }
    if (avail < 2)
        return -1;
    *count = (((unsigned)last << 8) | end[-2]) & 0x7fff;
    return 2;
}

inline int get_column_tail(const uint8_t* end, int avail, unsigned* column) // :405-427
{
    if (avail < 1)
        return -1;
    const uint8_t last = end[-1];
    const int width = last >> 6;
    if (width <= 1) {
        *column = last;
        return 1;
    }
    if (avail < width)
        return -1;
    if (width == 2)
        *column = (((unsigned)last << 8) | end[-2]) & 0x3fff;
    else
        *column = (((unsigned)last << 16) | ((unsigned)end[-2] << 8) | end[-3]) & 0x3fffff;
    return width;
}

/// Parses the footer at the end of `bytes` bytes; returns its size or -1.
inline int read_footer(const uint8_t* data, unsigned bytes, RowMeta* m) // :759-800
{
    unsigned left = bytes;
    const uint8_t* end = data + bytes;
    int w = get_count_tail(end, left, &m->sumCount);
    if (w < 0)
        return -1;
    left -= w;
    end -= w;
    m->sumCount += 1;
    w = get_column_tail(end, (int)left, &m->columnStart);
    if (w < 0)
        return -1;
    left -= w;
    end -= w;
    if (m->sumCount <= 1) {
        m->ldpcCount = 1;
        m->row = 0;
    } else {
        w = get_count_tail(end, left, &m->ldpcCount);
        if (w < 0)
            return -1;
        left -= w;
        end -= w;
        if (m->sumCount < m->ldpcCount)
            return -1;
        if (left < 1)
            return -1;
        m->row = end[-1];
        left -= 1;
    }
    return (int)(bytes - left);
}

} // namespace sgpu
