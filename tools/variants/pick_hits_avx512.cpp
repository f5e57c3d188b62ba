// tools/variants/pick_hits_avx512.cpp -- a MEASURED DEAD END, kept for the
// record; not built into libsiamese_amd.so.
//
// generate_matrix's LDPC picks of a row of <= 64 columns drawn on the host by
// AVX-512 (PCG jump-ahead, eight draws per instruction) instead of read from
// the cached offset lists (codedef.cpp ldpc_offsets).  Bit-exact (a
// self-check against the scalar draws ran at init), but slower on both hosts:
// generate_matrix 25-27 K vs 22-23 K ticks per decode on the Xeon build host
// (round 4) and 17.0-17.1 K vs 13.4-13.8 K on the MI355X box's EPYC 9575F
// (round 5, profiles/r5f_vector_picks_ab.txt).  It was reached through
// ldpc_pick_hits() in DecoderCore::generate_matrix.

#include <immintrin.h>
#include <cstdint>
#include <vector>

namespace sgpu {

const uint32_t* ldpc_offsets(unsigned row, unsigned n, unsigned* count);
constexpr unsigned kPairRate = 16;

namespace {

constexpr uint64_t kPcgMul = 6364136223846793005ULL;

// Jump-ahead of the PCG state: j steps from S give A^j S + inc G_j
// (G_0 = 0, G_{j+1} = A G_j + 1), for lanes j = 0..7 and the stride 8
struct PcgJump
{
    alignas(64) uint64_t a[8];
    alignas(64) uint64_t g[8];
    uint64_t a8 = 0, g8 = 0;
    PcgJump()
    {
        uint64_t A = 1, G = 0;
        for (unsigned j = 0; j < 8; ++j) {
            a[j] = A;
            g[j] = G;
            G = kPcgMul * G + 1;
            A *= kPcgMul;
        }
        a8 = A;
        g8 = G;
    }
};
const PcgJump g_jump;

__attribute__((target("avx512f,avx512dq,avx512vl,avx512bw"))) void
pick_hits_avx512(unsigned row, unsigned n, const uint32_t* pc, uint32_t lo, uint32_t span, uint64_t* hit1,
                 uint64_t* hitRx)
{
    const unsigned picks = 2 * ((n + kPairRate - 1) / kPairRate);
    const uint64_t inc = ((uint64_t)row << 1) | 1u;
    uint64_t S = (inc + n) * kPcgMul + inc;   // the state after Seed(row, n)
    const uint64_t stepG = inc * g_jump.g8;
    const __m512i A = _mm512_load_si512(g_jump.a);
    const __m512i IG = _mm512_mullo_epi64(_mm512_load_si512(g_jump.g), _mm512_set1_epi64((long long)inc));
    const __m256i N = _mm256_set1_epi32((int)n);
    const __m512d invN = _mm512_set1_pd(1.0 / (double)(n ? n : 1));
    const __m256i LO = _mm256_set1_epi32((int)lo), SPAN = _mm256_set1_epi32((int)span);
    const __m256i M63 = _mm256_set1_epi32(63);
    const __m512i ONE = _mm512_set1_epi64(1);
    __m512i acc = _mm512_setzero_si512();
    for (unsigned k = 0; k < picks; k += 8) {
        // the states before draws k .. k + 7, and XSH-RR of each
        const __m512i st = _mm512_add_epi64(_mm512_mullo_epi64(A, _mm512_set1_epi64((long long)S)), IG);
        S = S * g_jump.a8 + stepG;
        const __m512i xs = _mm512_srli_epi64(_mm512_xor_si512(_mm512_srli_epi64(st, 18), st), 27);
        const __m256i x = _mm256_rorv_epi32(_mm512_cvtepi64_epi32(xs), _mm512_cvtepi64_epi32(_mm512_srli_epi64(st, 59)));
        // x % n: a double-precision quotient (within one), corrected exactly
        const __m256i q = _mm512_cvttpd_epu32(_mm512_mul_pd(_mm512_cvtepu32_pd(x), invN));
        __m256i r = _mm256_sub_epi32(x, _mm256_mullo_epi32(q, N));
        r = _mm256_add_epi32(r, _mm256_and_si256(_mm256_srai_epi32(r, 31), N));
        r = _mm256_mask_sub_epi32(r, _mm256_cmpge_epu32_mask(r, N), r, N);
        const __mmask8 live = picks - k >= 8 ? (__mmask8)0xff : (__mmask8)((1u << (picks - k)) - 1u);
        const __m256i c = _mm256_mmask_i32gather_epi32(_mm256_setzero_si256(), live, r, pc, 4);
        const __mmask8 ok = _mm256_mask_cmplt_epu32_mask(live, _mm256_sub_epi32(c, LO), SPAN);
        acc = _mm512_xor_si512(acc, _mm512_maskz_sllv_epi64(ok, ONE, _mm512_cvtepu32_epi64(_mm256_and_si256(c, M63))));
    }
    alignas(64) uint64_t v[8];
    _mm512_store_si512(v, acc);
    *hit1 = v[0] ^ v[2] ^ v[4] ^ v[6];
    *hitRx = v[1] ^ v[3] ^ v[5] ^ v[7];
}

void pick_hits_scalar(unsigned row, unsigned n, const uint32_t* pc, uint32_t lo, uint32_t span, uint64_t* hit1,
                      uint64_t* hitRx)
{
    unsigned picks = 0;
    const uint32_t* off = ldpc_offsets(row, n, &picks);
    uint64_t h[2] = {0, 0};
    for (unsigned k = 0; k < picks; ++k) {
        const uint32_t c = pc[off[k]];
        h[k & 1] ^= (uint64_t)(c - lo < span) << (c & 63);
    }
    *hit1 = h[0];
    *hitRx = h[1];
}

// the vector draws where asked for, the host has AVX-512 DQ/VL and they
// reproduce the scalar sequence on a sweep of rows and window sizes
bool pick_hits_vector_ok()
{
    // (opt-in, SIAMESE_AMD_VECTOR_PICKS=1: on the Xeon build host the
    // cached offsets measured faster, 22-23K vs 25-27K ticks per generate)
    const char* v = std::getenv("SIAMESE_AMD_VECTOR_PICKS");
    if (!v || std::atoi(v) == 0)
        return false;
    if (!(__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
          __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512bw")))
        return false;
    std::vector<uint32_t> pc(70000);
    for (size_t i = 0; i < pc.size(); ++i)
        pc[i] = (uint32_t)((i * 2654435761u) >> 7) % 80u;
    const unsigned ns[] = {1, 2, 15, 16, 17, 63, 64, 200, 256, 257, 1000, 4096, 16000, 65535};
    for (unsigned row = 0; row < 256; row += 7)
        for (unsigned n : ns)
            for (uint32_t lo : {0u, 5u}) {
                uint64_t a0, a1, b0, b1;
                pick_hits_avx512(row, n, pc.data(), lo, 64 - lo - (row & 3), &a0, &a1);
                pick_hits_scalar(row, n, pc.data(), lo, 64 - lo - (row & 3), &b0, &b1);
                if (a0 != b0 || a1 != b1)
                    return false;
            }
    return true;
}

} // namespace

bool ldpc_pick_hits(unsigned row, unsigned n, const uint32_t* pc, uint32_t lo, uint32_t span, uint64_t* hit1,
                    uint64_t* hitRx)
{
    static const bool vec = pick_hits_vector_ok();
    if (!vec)
        return false;
    pick_hits_avx512(row, n, pc, lo, span, hit1, hitRx);
    return true;
}


} // namespace sgpu
