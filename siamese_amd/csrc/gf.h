// gf.h -- host-side GF(2^8) arithmetic for the control plane.
//
// Field: GF(2^8) modulo x^8+x^6+x^3+x^2+1 (0x14D), the polynomial the
// reference selects (reference gf256.cpp:357-372, index 3 of its table).
// The host only touches COEFFICIENTS (recovery-matrix generation and the
// Gaussian elimination on <=255x255 bytes); every symbol-sized operation is
// executed on the MI355X by the kernels in kernels.hip.
#pragma once

#include <cstdint>

namespace sgpu {

struct GfTables
{
    uint8_t exp[512 + 2];   // exp[i] = g^(i mod 255), doubled to skip a modulo
    uint16_t log[256];      // log[0] unused
    uint8_t mul[256][256];  // mul[y][x] = x*y
    uint8_t inv[256];       // inv[0] = 0
    uint8_t sqr[256];
    // Nibble tables for the AVX2 row kernel: lo[y][n] = y*n, hi[y][n] = y*(n<<4)
    alignas(32) uint8_t nib_lo[256][16];
    alignas(32) uint8_t nib_hi[256][16];
    // Multiply-by-y as the 8x8 bit matrix GF2P8AFFINEQB applies to every
    // byte: byte 7-i of affine[y] holds, in bit j, bit i of y * 2^j
    uint64_t affine[256];
};

extern GfTables g_gf;

/// Build the tables; idempotent.  Returns false if the self-check fails.
bool gf_init();

inline uint8_t gf_mul(uint8_t x, uint8_t y) { return g_gf.mul[y][x]; }
inline uint8_t gf_inv(uint8_t x) { return g_gf.inv[x]; }
inline uint8_t gf_sqr(uint8_t x) { return g_gf.sqr[x]; }
inline uint8_t gf_div(uint8_t x, uint8_t y) { return y ? g_gf.mul[g_gf.inv[y]][x] : 0; }

/// dst[i] ^= y * src[i] for i < n (host rows of the coefficient matrix).
/// The tail is done with a blended 32-byte vector, so both buffers must stay
/// readable and dst writable up to 31 bytes past n (bytes there are
/// rewritten unchanged).
void gf_muladd_row(uint8_t* dst, const uint8_t* src, uint8_t y, unsigned n);

/// A coefficient row segment split into nibbles once, for many
/// dst ^= y * src updates with the same src (one Gaussian-elimination pivot
/// row against every row below it): up to kGfRowMax bytes.
struct GfRowSrc
{
    static constexpr unsigned kGfRowMax = 288;   // align32(255 + 4) + slack
    alignas(32) uint8_t lo[kGfRowMax];
    alignas(32) uint8_t hi[kGfRowMax];
    unsigned n = 0;
};
/// Split src[0, n) (readable 31 bytes past n) into `out`; n <= kGfRowMax - 32.
void gf_row_prepare(GfRowSrc& out, const uint8_t* src, unsigned n);
/// dst[i] ^= y * src[i] for i < src.n with the prepared src (dst writable
/// 31 bytes past n, rewritten unchanged).
void gf_muladd_prepared(uint8_t* dst, const GfRowSrc& src, uint8_t y);

/// dst[i] ^= y * src[i] for i < n: GF2P8AFFINEQB over 64-byte masked
/// vectors where the host has GFNI and AVX-512BW (no slack past n needed;
/// one instruction multiplies 64 bytes by y), else gf_muladd_row.
extern void (*gf_muladd_fast)(uint8_t* dst, const uint8_t* src, uint8_t y, unsigned n);
/// True when gf_muladd_fast runs on GFNI.
bool gf_gfni();
/// Gaussian elimination without pivoting over rows [0, rows) of an m-column
/// matrix (row r at mat + r * stride, stride >= align(columns) + 64), the
/// reference's GaussianElimination loop (SiameseDecoder.cpp:2423-2466): for
/// pivot p = from, from + 1, ... while the pivot byte is non-zero, every row
/// below gets y = row[p] / pivot stored at [p] and y * pivot row (p, end[p])
/// added after it.  Returns the first pivot whose byte is zero (columns when
/// none is), with *bytes += the multiplied bytes (the reference's muladds).
/// GFNI + AVX-512 where the host has them (*done = false otherwise: the
/// caller runs its own loop).
unsigned gf_ge_nopivot(uint8_t* mat, unsigned stride, unsigned rows, unsigned columns, unsigned from,
                       const unsigned* end, uint64_t* bytes, bool* done);

/// Number of non-zero bytes in row[0, n) (AVX-512 where the host has it).
extern unsigned (*gf_count_nonzero)(const uint8_t* row, unsigned n);

/// Dense Siamese coefficients of one recovery row for `n` lost columns
/// (reference SiameseDecoder.cpp:2278-2300): out[j] = comb(opLo[lane[j]]) ^
/// RX * comb(opHi[lane[j]]) with comb(k) = (k&1) ^ (k&2 ? cx[j] : 0) ^
/// (k&4 ? cx2[j] : 0).  opLo/opHi: the row's opcode bits 0-2 / 3-5 per lane.
/// All arrays readable (out writable, rewritten unchanged) 31 bytes past n.
void gf_dense_row(uint8_t* out, const uint8_t* lane, const uint8_t* cx, const uint8_t* cx2,
                  const uint8_t opLo[8], const uint8_t opHi[8], uint8_t rx, unsigned n);

} // namespace sgpu
