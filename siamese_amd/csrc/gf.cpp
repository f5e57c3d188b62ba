// gf.cpp -- host GF(2^8) tables and the AVX2 coefficient-row kernel.
#include "gf.h"

#include <immintrin.h>
#include <cstdlib>
#include <cstring>

namespace sgpu {

GfTables g_gf;

static bool g_ready = false;

void gf_muladd_gfni(uint8_t* dst, const uint8_t* src, uint8_t y, unsigned n);
static unsigned count_nonzero_avx512(const uint8_t* row, unsigned n);

bool gf_init()
{
    if (g_ready)
        return true;

    // exp/log by repeated doubling modulo the field polynomial
    // (same field as reference gf256.cpp:379-403).
    const unsigned poly = 0x14D;
    unsigned v = 1;
    for (unsigned i = 0; i < 255; ++i) {
        g_gf.exp[i] = (uint8_t)v;
        g_gf.exp[i + 255] = (uint8_t)v;
        g_gf.log[v] = (uint16_t)i;
        v <<= 1;
        if (v & 0x100)
            v ^= poly;
    }
    g_gf.exp[510] = g_gf.exp[0];
    g_gf.exp[511] = g_gf.exp[1];
    g_gf.log[0] = 512;

    for (unsigned y = 0; y < 256; ++y) {
        for (unsigned x = 0; x < 256; ++x) {
            uint8_t p = 0;
            if (x && y)
                p = g_gf.exp[g_gf.log[x] + g_gf.log[y]];
            g_gf.mul[y][x] = p;
        }
    }
    g_gf.inv[0] = 0;
    for (unsigned x = 1; x < 256; ++x)
        g_gf.inv[x] = g_gf.exp[(255 - g_gf.log[x]) % 255];
    for (unsigned x = 0; x < 256; ++x)
        g_gf.sqr[x] = g_gf.mul[x][x];
    for (unsigned y = 0; y < 256; ++y) {
        for (unsigned n = 0; n < 16; ++n) {
            g_gf.nib_lo[y][n] = g_gf.mul[y][n];
            g_gf.nib_hi[y][n] = g_gf.mul[y][n << 4];
        }
    }

    for (unsigned y = 0; y < 256; ++y) {
        uint64_t m = 0;
        for (unsigned i = 0; i < 8; ++i) {
            unsigned row = 0;
            for (unsigned j = 0; j < 8; ++j)
                row |= ((g_gf.mul[y][1u << j] >> i) & 1u) << j;
            m |= (uint64_t)row << (8 * (7 - i));
        }
        g_gf.affine[y] = m;
    }
    if (__builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vl"))
        gf_count_nonzero = count_nonzero_avx512;
    if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw") &&
        __builtin_cpu_supports("avx512vl")) {
        gf_muladd_fast = gf_muladd_gfni;
        // the instruction against the tables, every y on every x
        alignas(64) uint8_t x[256], d[256];
        for (unsigned i = 0; i < 256; ++i)
            x[i] = (uint8_t)i;
        for (unsigned y = 0; y < 256; ++y) {
            std::memset(d, 0, sizeof(d));
            gf_muladd_gfni(d, x, (uint8_t)y, 256);
            for (unsigned i = 0; i < 256; ++i)
                if (d[i] != g_gf.mul[y][i])
                    return false;
        }
    }

    // Self-check: every non-zero element times its inverse is one, and the
    // known answers the reference pins.
    for (unsigned x = 1; x < 256; ++x)
        if (g_gf.mul[g_gf.inv[x]][x] != 1)
            return false;
    if (g_gf.mul[0x80][2] != 0x4d || g_gf.mul[0xca][0x53] != 0x94 || g_gf.inv[2] != 0xa6 ||
        g_gf.sqr[3] != 0x05)
        return false;

    g_ready = true;
    return true;
}

__attribute__((target("avx512f,avx512bw,avx512vl,gfni"))) void gf_muladd_gfni(uint8_t* dst, const uint8_t* src,
                                                                              uint8_t y, unsigned n)
{
    if (y == 0 || n == 0)
        return;
    const __m512i a = _mm512_set1_epi64((long long)g_gf.affine[y]);
    unsigned i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m512i x = _mm512_loadu_si512((const void*)(src + i));
        const __m512i d = _mm512_loadu_si512((const void*)(dst + i));
        _mm512_storeu_si512((void*)(dst + i), _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(x, a, 0)));
    }
    if (i < n) {
        const __mmask64 k = (1ull << (n - i)) - 1;   // (n - i < 64)
        const __m512i x = _mm512_maskz_loadu_epi8(k, src + i);
        const __m512i d = _mm512_maskz_loadu_epi8(k, dst + i);
        _mm512_mask_storeu_epi8(dst + i, k, _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(x, a, 0)));
    }
}

void (*gf_muladd_fast)(uint8_t*, const uint8_t*, uint8_t, unsigned) = gf_muladd_row;

__attribute__((target("avx512f,avx512bw,avx512vl,gfni"))) static unsigned ge_nopivot_gfni(
    uint8_t* mat, unsigned stride, unsigned rows, unsigned columns, unsigned from, const unsigned* end,
    uint64_t* bytes)
{
    uint64_t b = 0;
    unsigned p = from;
    for (; p < columns; ++p) {
        uint8_t* ge = mat + (size_t)p * stride;
        const uint8_t val = ge[p];
        if (val == 0)
            break;
        const unsigned n = end[p] > p + 1 ? end[p] - p - 1 : 0;
        const uint8_t* invRow = g_gf.mul[g_gf.inv[val]];
        // the pivot row's bytes after the pivot, in registers for every row below
        const unsigned chunks = (n + 63) / 64;
        __m512i src[4];
        __mmask64 km[4];
        for (unsigned c = 0; c < 4; ++c) {
            const unsigned lo = c * 64;
            km[c] = lo >= n ? 0 : (n - lo >= 64 ? ~0ull : (1ull << (n - lo)) - 1);
            src[c] = _mm512_maskz_loadu_epi8(km[c], ge + p + 1 + lo);
        }
        for (unsigned k = p + 1; k < rows; ++k) {
            uint8_t* row = mat + (size_t)k * stride;
            const uint8_t vj = row[p];
            if (vj == 0)
                continue;
            const uint8_t y = invRow[vj];
            row[p] = y;
            if (!n)
                continue;
            b += n;
            const __m512i a = _mm512_set1_epi64((long long)g_gf.affine[y]);
            for (unsigned c = 0; c < chunks; ++c) {
                uint8_t* d = row + p + 1 + c * 64;
                const __m512i x = _mm512_maskz_loadu_epi8(km[c], d);
                _mm512_mask_storeu_epi8(d, km[c], _mm512_xor_si512(x, _mm512_gf2p8affine_epi64_epi8(src[c], a, 0)));
            }
        }
    }
    *bytes += b;
    return p;
}

unsigned gf_ge_nopivot(uint8_t* mat, unsigned stride, unsigned rows, unsigned columns, unsigned from,
                       const unsigned* end, uint64_t* bytes, bool* done)
{
    *done = gf_gfni() && columns <= 256;
    return *done ? ge_nopivot_gfni(mat, stride, rows, columns, from, end, bytes) : from;
}

static unsigned count_nonzero_scalar(const uint8_t* row, unsigned n)
{
    unsigned c = 0;
    for (unsigned i = 0; i < n; ++i)
        c += row[i] != 0;
    return c;
}

__attribute__((target("avx512f,avx512bw,avx512vl"))) static unsigned count_nonzero_avx512(const uint8_t* row,
                                                                                        unsigned n)
{
    unsigned c = 0, i = 0;
    for (; i + 64 <= n; i += 64)
        c += (unsigned)__builtin_popcountll(
            _mm512_test_epi8_mask(_mm512_loadu_si512((const void*)(row + i)), _mm512_set1_epi8(-1)));
    if (i < n) {
        const __mmask64 k = (1ull << (n - i)) - 1;
        c += (unsigned)__builtin_popcountll(
            _mm512_mask_test_epi8_mask(k, _mm512_maskz_loadu_epi8(k, row + i), _mm512_set1_epi8(-1)));
    }
    return c;
}

unsigned (*gf_count_nonzero)(const uint8_t*, unsigned) = count_nonzero_scalar;

bool gf_gfni()
{
    return gf_muladd_fast == gf_muladd_gfni;
}

namespace {

// bytes [0, k) of a 32-byte vector selected (k in 1..32)
inline __m256i head_mask(unsigned k)
{
    const __m256i iota = _mm256_setr_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17,
                                          18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31);
    return _mm256_cmpgt_epi8(_mm256_set1_epi8((char)k), iota);
}

inline __m256i gf_mul32(__m256i x, __m256i tlo, __m256i thi)
{
    const __m256i m0f = _mm256_set1_epi8(0x0f);
    const __m256i lo = _mm256_and_si256(x, m0f);
    const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), m0f);
    return _mm256_xor_si256(_mm256_shuffle_epi8(tlo, lo), _mm256_shuffle_epi8(thi, hi));
}

} // namespace

void gf_muladd_row(uint8_t* dst, const uint8_t* src, uint8_t y, unsigned n)
{
    if (y == 0 || n == 0)
        return;
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_lo[y]));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_hi[y]));
    for (unsigned i = 0; i < n; i += 32) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(src + i));
        const __m256i d = _mm256_loadu_si256((const __m256i*)(dst + i));
        const __m256i p = y == 1 ? x : gf_mul32(x, tlo, thi);
        __m256i r = _mm256_xor_si256(d, p);
        if (n - i < 32)
            r = _mm256_blendv_epi8(d, r, head_mask(n - i));
        _mm256_storeu_si256((__m256i*)(dst + i), r);
    }
}

void gf_row_prepare(GfRowSrc& out, const uint8_t* src, unsigned n)
{
    const __m256i m0f = _mm256_set1_epi8(0x0f);
    out.n = n;
    for (unsigned i = 0; i < n; i += 32) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(src + i));
        _mm256_store_si256((__m256i*)(out.lo + i), _mm256_and_si256(x, m0f));
        _mm256_store_si256((__m256i*)(out.hi + i), _mm256_and_si256(_mm256_srli_epi64(x, 4), m0f));
    }
}

void gf_muladd_prepared(uint8_t* dst, const GfRowSrc& src, uint8_t y)
{
    const unsigned n = src.n;
    if (y == 0 || n == 0)
        return;
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_lo[y]));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_hi[y]));
    for (unsigned i = 0; i < n; i += 32) {
        const __m256i p = _mm256_xor_si256(
            _mm256_shuffle_epi8(tlo, _mm256_load_si256((const __m256i*)(src.lo + i))),
            _mm256_shuffle_epi8(thi, _mm256_load_si256((const __m256i*)(src.hi + i))));
        const __m256i d = _mm256_loadu_si256((const __m256i*)(dst + i));
        __m256i r = _mm256_xor_si256(d, p);
        if (n - i < 32)
            r = _mm256_blendv_epi8(d, r, head_mask(n - i));
        _mm256_storeu_si256((__m256i*)(dst + i), r);
    }
}

void gf_dense_row(uint8_t* out, const uint8_t* lane, const uint8_t* cx, const uint8_t* cx2,
                  const uint8_t opLo[8], const uint8_t opHi[8], uint8_t rx, unsigned n)
{
    uint8_t lo16[16] = {0}, hi16[16] = {0};
    for (unsigned l = 0; l < 8; ++l) {
        lo16[l] = opLo[l];
        hi16[l] = opHi[l];
    }
    const __m256i tLo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)lo16));
    const __m256i tHi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)hi16));
    const __m256i rlo = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_lo[rx]));
    const __m256i rhi = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_hi[rx]));
    const __m256i one = _mm256_set1_epi8(1), two = _mm256_set1_epi8(2), four = _mm256_set1_epi8(4);
    // comb(k) for the selector vector k
    auto comb = [&](__m256i k, __m256i c1, __m256i c2) {
        const __m256i b0 = _mm256_and_si256(k, one);
        const __m256i b1 = _mm256_cmpeq_epi8(_mm256_and_si256(k, two), two);
        const __m256i b2 = _mm256_cmpeq_epi8(_mm256_and_si256(k, four), four);
        return _mm256_xor_si256(b0, _mm256_xor_si256(_mm256_and_si256(b1, c1), _mm256_and_si256(b2, c2)));
    };
    for (unsigned j = 0; j < n; j += 32) {
        const __m256i L = _mm256_loadu_si256((const __m256i*)(lane + j));
        const __m256i c1 = _mm256_loadu_si256((const __m256i*)(cx + j));
        const __m256i c2 = _mm256_loadu_si256((const __m256i*)(cx2 + j));
        const __m256i v = _mm256_xor_si256(comb(_mm256_shuffle_epi8(tLo, L), c1, c2),
                                           gf_mul32(comb(_mm256_shuffle_epi8(tHi, L), c1, c2), rlo, rhi));
        __m256i r = v;
        if (n - j < 32)
            r = _mm256_blendv_epi8(_mm256_loadu_si256((const __m256i*)(out + j)), v, head_mask(n - j));
        _mm256_storeu_si256((__m256i*)(out + j), r);
    }
}

} // namespace sgpu
