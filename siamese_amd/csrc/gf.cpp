// gf.cpp -- host GF(2^8) tables and the AVX2 coefficient-row kernel.
#include "gf.h"

#include <immintrin.h>
#include <cstring>

namespace sgpu {

GfTables g_gf;

static bool g_ready = false;

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

void gf_muladd_row(uint8_t* dst, const uint8_t* src, uint8_t y, unsigned n)
{
    if (y == 0 || n == 0)
        return;
    unsigned i = 0;
    if (y == 1) {
        for (; i + 32 <= n; i += 32) {
            __m256i a = _mm256_loadu_si256((const __m256i*)(dst + i));
            __m256i b = _mm256_loadu_si256((const __m256i*)(src + i));
            _mm256_storeu_si256((__m256i*)(dst + i), _mm256_xor_si256(a, b));
        }
        for (; i < n; ++i)
            dst[i] ^= src[i];
        return;
    }
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_lo[y]));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)g_gf.nib_hi[y]));
    const __m256i m0f = _mm256_set1_epi8(0x0f);
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i*)(src + i));
        __m256i lo = _mm256_and_si256(x, m0f);
        __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), m0f);
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, lo), _mm256_shuffle_epi8(thi, hi));
        __m256i d = _mm256_loadu_si256((const __m256i*)(dst + i));
        _mm256_storeu_si256((__m256i*)(dst + i), _mm256_xor_si256(d, p));
    }
    const uint8_t* row = g_gf.mul[y];
    for (; i < n; ++i)
        dst[i] ^= row[src[i]];
}

} // namespace sgpu
