// tools/gf_mul_bench.hip -- A/B of the GF(256) multiply-by-constant
// primitives a solve sweep can use on gfx950 (profiling aid, not shipped):
//   perm    three v_perm_b32 lookups per dword (bits 0-2, 3-5, 6-7 of each
//           byte; the product tables of y in registers) -- the product's choice
//   logexp  log/exp tables in LDS (reference gf256.cpp:379-403): per byte one
//           log lookup of the source and one exp lookup of the sum
//   mulrow  the 256-byte product row of y in LDS: one lookup per byte
// Each kernel computes dst ^= sum_k (y + k) * src, k < Y, over `bytes`
// bytes with a per-block base y, 16 bytes per lane (the solve's tile width):
// Y = 16 or 64 multiplies per loaded byte, as a solve multiplies one source
// row into many output rows; at 64 the multiply -- not HBM -- sets the time.
// The host checks every byte.  Prints products per second per primitive
// (median of 5 timed launches).
//   hipcc --offload-arch=gfx950 -O3 -o tools/gf_mul_bench tools/gf_mul_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

uint8_t g_exp[512], g_log[256], g_mul[256][256];

void tables()
{
    // GF(2^8) modulo 0x14D (reference gf256.cpp:357-372), generator 2
    unsigned x = 1;
    for (unsigned i = 0; i < 255; ++i) {
        g_exp[i] = g_exp[i + 255] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100)
            x ^= 0x14D;
    }
    g_exp[510] = g_exp[511] = 0;
    for (unsigned a = 0; a < 256; ++a)
        for (unsigned b = 0; b < 256; ++b)
            g_mul[a][b] = (a && b) ? g_exp[g_log[a] + g_log[b]] : 0;
}

__constant__ uint32_t c_perm[256][8];
__constant__ uint8_t c_exp[512];
__constant__ uint8_t c_log[256];
__constant__ uint8_t c_mul[256][256];

__device__ __forceinline__ uint32_t perm_mul(uint32_t x, uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                             uint32_t c)
{
    return __builtin_amdgcn_perm(a1, a0, x & 0x07070707u) ^ __builtin_amdgcn_perm(b1, b0, (x >> 3) & 0x07070707u) ^
           __builtin_amdgcn_perm(0u, c, (x >> 6) & 0x03030303u);
}

template <uint32_t kY>
__global__ __launch_bounds__(256) void k_perm(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16)
{
    const uint32_t y0 = (blockIdx.x * 97u + 13u) & 255u;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256u) {
        const uint4 s = src[i];
        uint4 d = dst[i];
#pragma unroll
        for (uint32_t k = 0; k < kY; ++k) {
            const uint32_t* t = c_perm[(y0 + k) & 255u];
            const uint32_t a0 = t[0], a1 = t[1], b0 = t[2], b1 = t[3], c = t[4];
            d.x ^= perm_mul(s.x, a0, a1, b0, b1, c);
            d.y ^= perm_mul(s.y, a0, a1, b0, b1, c);
            d.z ^= perm_mul(s.z, a0, a1, b0, b1, c);
            d.w ^= perm_mul(s.w, a0, a1, b0, b1, c);
        }
        dst[i] = d;
    }
}

__device__ __forceinline__ uint32_t logexp_mul(uint32_t x, uint32_t ly, const uint8_t* L, const uint8_t* E)
{
    uint32_t r = 0;
#pragma unroll
    for (unsigned k = 0; k < 4; ++k) {
        const uint32_t b = (x >> (8 * k)) & 255u;
        const uint32_t v = b ? E[L[b] + ly] : 0u;
        r |= v << (8 * k);
    }
    return r;
}

template <uint32_t kY>
__global__ __launch_bounds__(256) void k_logexp(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16)
{
    __shared__ uint8_t L[256], E[512];
    for (uint32_t k = threadIdx.x; k < 512; k += 256) {
        E[k] = c_exp[k];
        if (k < 256)
            L[k] = c_log[k];
    }
    __syncthreads();
    const uint32_t y0 = (blockIdx.x * 97u + 13u) & 255u;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256u) {
        const uint4 s = src[i];
        uint4 d = dst[i];
#pragma unroll
        for (uint32_t k = 0; k < kY; ++k) {
            const uint32_t y = (y0 + k) & 255u;
            if (!y)
                continue;
            const uint32_t ly = c_log[y];
            d.x ^= logexp_mul(s.x, ly, L, E);
            d.y ^= logexp_mul(s.y, ly, L, E);
            d.z ^= logexp_mul(s.z, ly, L, E);
            d.w ^= logexp_mul(s.w, ly, L, E);
        }
        dst[i] = d;
    }
}

__device__ __forceinline__ uint32_t row_mul(uint32_t x, const uint8_t* M)
{
    return (uint32_t)M[x & 255u] | (uint32_t)M[(x >> 8) & 255u] << 8 | (uint32_t)M[(x >> 16) & 255u] << 16 |
           (uint32_t)M[x >> 24] << 24;
}

template <uint32_t kY>
__global__ __launch_bounds__(256) void k_mulrow(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16)
{
    __shared__ uint8_t M[kY][256];
    const uint32_t y0 = (blockIdx.x * 97u + 13u) & 255u;
    for (uint32_t k = 0; k < kY; ++k)
        M[k][threadIdx.x] = c_mul[(y0 + k) & 255u][threadIdx.x];   // (kY x 256 B of LDS)
    __syncthreads();
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256u) {
        const uint4 s = src[i];
        uint4 d = dst[i];
#pragma unroll
        for (uint32_t k = 0; k < kY; ++k) {
            d.x ^= row_mul(s.x, M[k]);
            d.y ^= row_mul(s.y, M[k]);
            d.z ^= row_mul(s.z, M[k]);
            d.w ^= row_mul(s.w, M[k]);
        }
        dst[i] = d;
    }
}

#define CK(x)                                                                       \
    do {                                                                            \
        if ((x) != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(x));      \
            return 1;                                                               \
        }                                                                           \
    } while (0)

} // namespace

int main()
{
    tables();
    uint32_t perm[256][8] = {};
    for (unsigned y = 0; y < 256; ++y) {
        uint8_t lo[8], mid[8], hi[4];
        for (unsigned k = 0; k < 8; ++k) {
            lo[k] = g_mul[y][k];
            mid[k] = g_mul[y][k << 3];
        }
        for (unsigned k = 0; k < 4; ++k)
            hi[k] = g_mul[y][k << 6];
        std::memcpy(&perm[y][0], lo, 8);
        std::memcpy(&perm[y][2], mid, 8);
        std::memcpy(&perm[y][4], hi, 4);
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_perm), perm, sizeof(perm)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_exp), g_exp, sizeof(g_exp)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_log), g_log, sizeof(g_log)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_mul), g_mul, sizeof(g_mul)));

    const size_t bytes = 256u << 20, n16 = bytes / 16;
    std::vector<uint8_t> hs(bytes), hd(bytes), out(bytes);
    for (size_t i = 0; i < bytes; ++i) {
        hs[i] = (uint8_t)(i * 2654435761u >> 13);
        hd[i] = (uint8_t)(i * 40503u >> 7);
    }
    uint4 *src = nullptr, *dst = nullptr;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMemcpy(src, hs.data(), bytes, hipMemcpyHostToDevice));
    const unsigned blocks = 256u * 16u;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[3] = {"perm", "logexp", "mulrow"};
    for (uint32_t Y : {16u, 64u})
    for (int kind = 0; kind < 3; ++kind) {
        // correctness: one launch from a known dst
        CK(hipMemcpy(dst, hd.data(), bytes, hipMemcpyHostToDevice));
        auto launch = [&]() {
            if (kind == 0)
                {
                if (Y == 16)
                    hipLaunchKernelGGL(k_perm<16>, dim3(blocks), dim3(256), 0, 0, src, dst, n16);
                else
                    hipLaunchKernelGGL(k_perm<64>, dim3(blocks), dim3(256), 0, 0, src, dst, n16);
            }
            else if (kind == 1)
                {
                if (Y == 16)
                    hipLaunchKernelGGL(k_logexp<16>, dim3(blocks), dim3(256), 0, 0, src, dst, n16);
                else
                    hipLaunchKernelGGL(k_logexp<64>, dim3(blocks), dim3(256), 0, 0, src, dst, n16);
            }
            else
                {
                if (Y == 16)
                    hipLaunchKernelGGL(k_mulrow<16>, dim3(blocks), dim3(256), 0, 0, src, dst, n16);
                else
                    hipLaunchKernelGGL(k_mulrow<64>, dim3(blocks), dim3(256), 0, 0, src, dst, n16);
            }
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(out.data(), dst, bytes, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < bytes; ++i) {
            const size_t lanei = i / 16;
            const unsigned blk = (unsigned)((lanei / 256) % blocks);
            const unsigned y0 = (blk * 97u + 13u) & 255u;
            uint8_t want = hd[i];
            for (unsigned k = 0; k < Y; ++k)
                want ^= g_mul[(y0 + k) & 255u][hs[i]];
            if (out[i] != want)
                ++bad;
        }
        std::vector<float> ms;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r)
                ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double t = ms[ms.size() / 2];
        std::printf("%-7s Y=%-3u %8.3f ms per pass over %zu MiB: %7.1f G byte-products/s "
                    "(HBM %6.1f GB/s), %zu wrong bytes\n",
                    names[kind], Y, t, bytes >> 20, (double)Y * bytes / t / 1e6, 3.0 * bytes / t / 1e6, bad);
    }
    return 0;
}
