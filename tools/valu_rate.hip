// tools/valu_rate.hip -- issue rate of the VALU instructions the GF(256)
// multiply uses on gfx950 (profiling aid, not shipped): eight independent
// chains per lane of v_perm_b32, of v_xor_b32, and of the multiply's mix
// and of v_bitop3_b32 (three-way XOR), enough waves to fill every SIMD.
// Prints wave-instructions per SIMD-cycle at the measured clock-free rate:
// ns per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_perm(unsigned* out, unsigned seed)
{
    unsigned a[8], s0 = seed + threadIdx.x, s1 = seed * 3u + 7u;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        a[k] = seed ^ (threadIdx.x * (k + 1));
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[k]) : "v"(s0), "v"(s1));
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        r ^= a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_xor(unsigned* out, unsigned seed)
{
    unsigned a[8], s0 = seed + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        a[k] = seed ^ (threadIdx.x * (k + 1));
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[k]) : "v"(s0));
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        r ^= a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_perm_s(unsigned* out, unsigned seed)
{
    // v_perm_b32 with one SGPR table operand (the solve's form)
    unsigned a[8], s1 = seed * 3u + 7u;
    const unsigned s0 = __builtin_amdgcn_readfirstlane(seed * 5u + 1u);
#pragma unroll
    for (int k = 0; k < 8; ++k)
        a[k] = seed ^ (threadIdx.x * (k + 1));
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[k]) : "s"(s0), "v"(s1));
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        r ^= a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_bitop3(unsigned* out, unsigned seed)
{
    unsigned a[8], s0 = seed + threadIdx.x, s1 = seed * 3u + 7u;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        a[k] = seed ^ (threadIdx.x * (k + 1));
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[k]) : "v"(s0), "v"(s1));
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        r ^= a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main()
{
    unsigned* out = nullptr;
    const unsigned blocks = 256 * 4 * 8;   // 8 waves per SIMD over 256 CUs
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess)
        return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[4] = {"v_perm_b32 (vgpr)", "v_xor_b32", "v_perm_b32 (sgpr)", "v_bitop3_b32"};
    for (int kind = 0; kind < 4; ++kind) {
        float best = 1e9f;
        for (int r = 0; r < 5; ++r) {
            (void)hipEventRecord(e0, 0);
            if (kind == 0)
                hipLaunchKernelGGL(k_perm, dim3(blocks), dim3(256), 0, 0, out, 1u + r);
            else if (kind == 1)
                hipLaunchKernelGGL(k_xor, dim3(blocks), dim3(256), 0, 0, out, 1u + r);
            else if (kind == 2)
                hipLaunchKernelGGL(k_perm_s, dim3(blocks), dim3(256), 0, 0, out, 1u + r);
            else
                hipLaunchKernelGGL(k_bitop3, dim3(blocks), dim3(256), 0, 0, out, 1u + r);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (r && t < best)
                best = t;
        }
        // wave-instructions per SIMD: blocks * 4 waves * iters * 8 / 1024 SIMDs
        const double per = (double)blocks * 4 * kIters * 8 / 1024.0;
        std::printf("%-18s %8.3f ms  %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.4 GHz)\n", names[kind],
                    best, best * 1e6 / per, best * 1e6 / per * 2.4);
    }
    return 0;
}
