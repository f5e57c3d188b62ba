// tools/ge_microbench.cpp -- the coefficient elimination's row update in
// isolation: Gaussian elimination without pivoting over an m x m matrix of
// random GF(256) bytes, with the AVX2 nibble path (rows split once per
// pivot) and with GF2P8AFFINEQB (gf.h gf_muladd_fast).  Minimum of many
// trials, so a noisy host still gives a usable A/B.
//   g++ -O2 -mavx2 -std=c++17 -I siamese_amd/csrc tools/ge_microbench.cpp siamese_amd/csrc/gf.cpp -o /tmp/ge_mb
#include "gf.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace sgpu;

static double run(unsigned m, bool gfni, const std::vector<uint8_t>& init, unsigned stride, uint64_t* check)
{
    std::vector<uint8_t> mat(init);
    GfRowSrc src;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned p = 0; p < m; ++p) {
        const uint8_t* ge = mat.data() + (size_t)p * stride;
        const uint8_t val = ge[p];
        if (!val)
            continue;
        const unsigned n = m - p - 1;
        if (!gfni && n)
            gf_row_prepare(src, ge + p + 1, n);
        for (unsigned k = p + 1; k < m; ++k) {
            uint8_t* r = mat.data() + (size_t)k * stride;
            const uint8_t vj = r[p];
            if (!vj)
                continue;
            const uint8_t y = gf_div(vj, val);
            r[p] = y;
            if (!n)
                continue;
            if (gfni)
                gf_muladd_fast(r + p + 1, ge + p + 1, y, n);
            else
                gf_muladd_prepared(r + p + 1, src, y);
        }
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    uint64_t h = 1469598103934665603ULL;
    for (unsigned i = 0; i < m; ++i)
        for (unsigned j = 0; j < m; ++j)
            h = (h ^ mat[(size_t)i * stride + j]) * 1099511628211ULL;
    *check = h;
    return us;
}

int main(int argc, char** argv)
{
    if (!gf_init()) {
        std::fprintf(stderr, "gf_init failed\n");
        return 1;
    }
    const unsigned m = argc > 1 ? (unsigned)std::atoi(argv[1]) : 51;
    const unsigned trials = argc > 2 ? (unsigned)std::atoi(argv[2]) : 2000;
    const unsigned stride = argc > 3 ? (unsigned)std::atoi(argv[3]) : ((m + 4 + 31) / 32) * 32 + 32;
    std::mt19937 rng(7);
    std::vector<uint8_t> init((size_t)(m + 1) * stride, 0);
    for (unsigned i = 0; i < m; ++i)
        for (unsigned j = 0; j < m; ++j)
            init[(size_t)i * stride + j] = (uint8_t)(rng() % 255 + 1);
    std::printf("GE m=%u: gfni available %d\n", m, (int)gf_gfni());
    uint64_t ha = 0, hb = 0;
    double best[2] = {1e30, 1e30};
    for (unsigned t = 0; t < trials; ++t)
        for (int g = 0; g < 2; ++g) {
            if (g && !gf_gfni())
                continue;
            const double us = run(m, g != 0, init, stride, g ? &hb : &ha);
            if (us < best[g])
                best[g] = us;
        }
    std::printf("  avx2 nibbles %.2f us   gfni %.2f us   results equal %d\n", best[0], best[1],
                (int)(!gf_gfni() || ha == hb));
    return 0;
}
