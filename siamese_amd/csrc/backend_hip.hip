// backend_hip.hip -- gfx950 kernels and the HIP side of backend.h.
//
// Kernels (all byte-column local, see ops.h):
//   k_ingest       copy symbols (with their length prefix) into fresh buffers
//   k_exec         run one segment of every instance's op list on one 1 KiB
//                  tile: LINCOMB = XOR / GF(256) multiply-accumulate of up to
//                  thousands of source symbols into one destination
//   k_solve_prefix solve bytes 0..3 of every row of each triangular system
//                  (one wave per solve) to learn the recovered lengths
//   k_solve_main   lower-triangle multiply + back-substitution per tile
//
// GF(256) multiply by a wave-uniform constant uses three v_perm_b32 byte
// lookups per dword (bits 0-2, 3-5, 6-7 of each byte); the 32-byte table per
// constant lives in constant memory.  HBM traffic, not VALU, is the roofline.
#include <hip/hip_runtime.h>

#include "backend.h"
#include "gf.h"

#include <cstdio>
#include <cstring>
#include <vector>

namespace sgpu {

// ---------------------------------------------------------------------------
// Device tables

__constant__ uint32_t c_perm[256][8];   // per constant y: {Ta0,Ta1,Tb0,Tb1,Tc,0,0,0}
__constant__ uint8_t c_inv[256];

__device__ __forceinline__ uint32_t gf_mul_dword(uint32_t x, uint32_t y)
{
    const uint32_t* t = c_perm[y];
    const uint32_t a = x & 0x07070707u;
    const uint32_t b = (x >> 3) & 0x07070707u;
    const uint32_t c = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(t[1], t[0], a) ^ __builtin_amdgcn_perm(t[3], t[2], b) ^
           __builtin_amdgcn_perm(0u, t[4], c);
}

__device__ __forceinline__ uint4 gf_mul16(uint4 v, uint32_t y)
{
    uint4 r;
    r.x = gf_mul_dword(v.x, y);
    r.y = gf_mul_dword(v.y, y);
    r.z = gf_mul_dword(v.z, y);
    r.w = gf_mul_dword(v.w, y);
    return r;
}

__device__ __forceinline__ uint32_t byte_mask(int n)
{
    // mask of the low n bytes of a dword, n clamped to [0,4]
    return n <= 0 ? 0u : (n >= 4 ? 0xffffffffu : ((1u << (8 * n)) - 1u));
}

__device__ __forceinline__ uint4 mask16(uint4 v, int nbytes)
{
    v.x &= byte_mask(nbytes);
    v.y &= byte_mask(nbytes - 4);
    v.z &= byte_mask(nbytes - 8);
    v.w &= byte_mask(nbytes - 12);
    return v;
}

__device__ __forceinline__ uint4 xor16(uint4 a, uint4 b)
{
    return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__device__ __forceinline__ uint4 ld16(uint64_t addr)
{
    return *reinterpret_cast<const uint4*>(addr);
}

__device__ __forceinline__ void st16(uint64_t addr, uint4 v)
{
    *reinterpret_cast<uint4*>(addr) = v;
}

// ---------------------------------------------------------------------------
// Ingest

__global__ __launch_bounds__(64) void k_ingest(const IngestDesc* descs, const IngestItem* items)
{
    const IngestItem it = items[blockIdx.x];
    const IngestDesc d = descs[it.desc];
    const uint32_t total = d.hdrLen + d.bytes;
    const uint32_t p = it.tileBase + threadIdx.x * 16;
    if (p >= total)
        return;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
    uint8_t* dst = reinterpret_cast<uint8_t*>(d.dst);
    const uint64_t shifted = d.src - d.hdrLen; // address that lines up with dst
    if (p >= d.hdrLen && p + 16 <= total && (shifted & 15u) == 0) {
        st16((uint64_t)(dst + p), ld16(shifted + p));
        return;
    }
    const uint32_t end = p + 16 < total ? p + 16 : total;
    for (uint32_t k = p; k < end; ++k)
        dst[k] = k < d.hdrLen ? d.hdr[k] : src[k - d.hdrLen];
}

// ---------------------------------------------------------------------------
// Executor

__global__ __launch_bounds__(64) void k_exec(const GfOp* __restrict__ ops,
                                             const GfTerm* __restrict__ terms,
                                             const ExecItem* __restrict__ items)
{
    const ExecItem it = items[blockIdx.x];
    const uint32_t p = it.tileBase + threadIdx.x * 16;

    for (uint32_t oi = 0; oi < it.opCount; ++oi) {
        const GfOp op = ops[it.opBegin + oi];
        if (op.kind == OP_LITERAL) {
            const uint32_t a = op.n, b = op.n + op.valid;
            if (b <= p || a >= p + 16)
                continue;
            uint8_t* dst = reinterpret_cast<uint8_t*>(op.dst);
            for (uint32_t k = (a > p ? a : p); k < b && k < p + 16; ++k)
                dst[k] = op.lit[k - a];
            continue;
        }
        if (p >= op.n)
            continue;

        uint4 acc0 = make_uint4(0, 0, 0, 0);
        uint4 acc1 = make_uint4(0, 0, 0, 0);
        const GfTerm* t = terms + op.termBegin;
        const uint32_t nt = op.termCount;
        uint32_t k = 0;
        // Issue loads for 4 terms at a time so several HBM requests are in
        // flight per lane before the first XOR consumes one.
        for (; k + 4 <= nt; k += 4) {
            GfTerm tt[4];
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                tt[u] = t[k + u];
                v[u] = p < tt[u].len ? ld16(tt[u].src + p) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint4 x = v[u];
                if (p + 16 > tt[u].len)
                    x = mask16(x, (int)tt[u].len - (int)p);
                if (tt[u].coeff != 1)
                    x = gf_mul16(x, tt[u].coeff);
                if (tt[u].acc)
                    acc1 = xor16(acc1, x);
                else
                    acc0 = xor16(acc0, x);
            }
        }
        for (; k < nt; ++k) {
            const GfTerm tm = t[k];
            if (p >= tm.len)
                continue;
            uint4 x = ld16(tm.src + p);
            if (p + 16 > tm.len)
                x = mask16(x, (int)tm.len - (int)p);
            if (tm.coeff != 1)
                x = gf_mul16(x, tm.coeff);
            if (tm.acc)
                acc1 = xor16(acc1, x);
            else
                acc0 = xor16(acc0, x);
        }
        if (op.mix > 1)
            acc1 = gf_mul16(acc1, op.mix);
        uint4 out = xor16(acc0, acc1);
        if (p < op.valid) {
            uint4 prior = ld16(op.dst + p);
            if (p + 16 > op.valid)
                prior = mask16(prior, (int)op.valid - (int)p);
            out = xor16(out, prior);
        }
        if (p + 16 > op.n) {
            // keep dst bytes at and beyond n
            const int nb = (int)op.n - (int)p;
            const uint4 old = ld16(op.dst + p);
            const uint4 keep = make_uint4(~byte_mask(nb), ~byte_mask(nb - 4), ~byte_mask(nb - 8),
                                          ~byte_mask(nb - 12));
            out = mask16(out, nb);
            out.x |= old.x & keep.x;
            out.y |= old.y & keep.y;
            out.z |= old.z & keep.z;
            out.w |= old.w & keep.w;
        }
        st16(op.dst + p, out);
    }
}

// ---------------------------------------------------------------------------
// Triangular solve

__device__ __forceinline__ uint32_t ld4_masked(uint64_t addr, uint32_t bytes)
{
    // first four bytes of a row, bytes at/after `bytes` read as zero
    const uint32_t v = *reinterpret_cast<const uint32_t*>(addr);
    return v & byte_mask((int)bytes);
}

// Length prefix parser (reference SiameseSerializers.h:596-627) on 4 bytes.
__device__ __forceinline__ int parse_prefix(uint32_t w, uint32_t avail, uint32_t* len)
{
    const uint32_t b0 = w & 0xff, b1 = (w >> 8) & 0xff, b2 = (w >> 16) & 0xff, b3 = w >> 24;
    if (avail < 1)
        return -1;
    const uint32_t top = b0 >> 6;
    if (top <= 1) {
        *len = b0;
        return 1;
    }
    if (top == 2) {
        if (avail < 2)
            return -1;
        *len = ((b0 << 8) | b1) & 0x3fff;
        return 2;
    }
    if ((b0 & 0xE0) == 0xC0) {
        if (avail < 3)
            return -1;
        *len = ((b0 << 16) | (b1 << 8) | b2) & 0x1fffff;
        return 3;
    }
    if (avail < 4)
        return -1;
    *len = ((b0 << 24) | (b1 << 16) | (b2 << 8) | b3) & 0x1fffffff;
    return 4;
}

__global__ __launch_bounds__(64) void k_solve_prefix(const SolveDesc* __restrict__ solves,
                                                     const SolveRow* __restrict__ rows,
                                                     const uint8_t* __restrict__ coef,
                                                     uint32_t* __restrict__ results)
{
    __shared__ uint32_t P[256];
    __shared__ uint32_t X;
    __shared__ uint32_t bb;
    __shared__ int stop;
    const SolveDesc sd = solves[blockIdx.x];
    const uint32_t m = sd.m;
    const SolveRow* R = rows + sd.rowBegin;
    const uint8_t* C = coef + sd.coefOffset;
    uint32_t* out = results + sd.result;
    const uint32_t lane = threadIdx.x;

    for (uint32_t j = lane; j < m; j += 64)
        P[j] = ld4_masked(R[j].buf, R[j].initBytes);
    if (lane == 0)
        stop = 0;
    __syncthreads();

    // MultiplyLowerTriangle on bytes 0..3 (reference SiameseDecoder.cpp:1065-1104)
    for (uint32_t i = 0; i + 1 < m; ++i) {
        const uint32_t src = P[i] & byte_mask((int)R[i].lowerLen);
        for (uint32_t j = i + 1 + lane; j < m; j += 64) {
            const uint32_t y = C[(size_t)j * m + i];
            if (y)
                P[j] ^= gf_mul_dword(src, y);
        }
        __syncthreads();
    }

    // BackSubstitution on bytes 0..3 (reference SiameseDecoder.cpp:1106-1238)
    uint32_t ok = 0;
    for (int i = (int)m - 1; i >= 0; --i) {
        if (lane == 0) {
            const uint32_t fb = R[i].finalBytes;
            const uint32_t lc = fb < 32 ? fb : 32;
            const uint32_t y = C[(size_t)i * m + i];
            const uint32_t x = gf_mul_dword(P[i], c_inv[y]) & byte_mask((int)lc);
            uint32_t len = 0;
            const int h = parse_prefix(x, lc, &len);
            if (h < 1 || len == 0 || (uint32_t)h + len > fb) {
                stop = 1;
            } else {
                out[1 + i] = ((uint32_t)h << 29) | len;
                bb = (uint32_t)h + len;
                X = x & byte_mask((int)bb);
            }
        }
        __syncthreads();
        if (stop)
            break;
        ++ok;
        const uint32_t xi = X, b = bb;
        for (uint32_t j = lane; j < (uint32_t)i; j += 64) {
            const uint32_t c = C[(size_t)j * m + i];
            if (c) {
                const uint32_t ab = b < R[j].finalBytes ? b : R[j].finalBytes;
                P[j] ^= gf_mul_dword(xi & byte_mask((int)ab), c);
            }
        }
        __syncthreads();
    }
    if (lane == 0)
        out[0] = ok;
}

__global__ __launch_bounds__(64) void k_solve_main(const SolveDesc* __restrict__ solves,
                                                   const SolveRow* __restrict__ rows,
                                                   const uint8_t* __restrict__ coef,
                                                   const uint32_t* __restrict__ results,
                                                   const SolveItem* __restrict__ items)
{
    const SolveItem it = items[blockIdx.x];
    const SolveDesc sd = solves[it.solve];
    const uint32_t m = sd.m;
    const SolveRow* R = rows + sd.rowBegin;
    const uint8_t* C = coef + sd.coefOffset;
    const uint32_t* res = results + sd.result;
    const uint32_t p = it.tileBase + threadIdx.x * 16;
    if (p >= sd.maxBytes)
        return;

    // Zero the region each row grows into (GrowZeroPadded) up front.
    for (uint32_t j = 0; j < m; ++j) {
        const uint32_t a = R[j].initBytes, b = R[j].finalBytes;
        if (b <= a || p >= b || p + 16 <= a)
            continue;
        uint4 v = ld16(R[j].buf + p);
        const uint4 keep = mask16(make_uint4(~0u, ~0u, ~0u, ~0u), (int)a - (int)p);
        v.x &= keep.x;
        v.y &= keep.y;
        v.z &= keep.z;
        v.w &= keep.w;
        st16(R[j].buf + p, v);
    }

    // Lower triangle in pivot order
    for (uint32_t i = 0; i + 1 < m; ++i) {
        const uint32_t L = R[i].lowerLen;
        if (p >= L)
            continue;
        uint4 src = ld16(R[i].buf + p);
        if (p + 16 > L)
            src = mask16(src, (int)L - (int)p);
        for (uint32_t j = i + 1; j < m; ++j) {
            const uint32_t y = C[(size_t)j * m + i];
            if (!y)
                continue;
            st16(R[j].buf + p, xor16(ld16(R[j].buf + p), gf_mul16(src, y)));
        }
    }

    // Back-substitution from the right-most column
    const uint32_t ok = res[0];
    for (int i = (int)m - 1; i >= 0; --i) {
        if ((uint32_t)(m - 1 - i) >= ok)
            break;
        const uint32_t w = res[1 + i];
        const uint32_t bb = (w >> 29) + (w & kSolveLengthMask);
        const uint32_t fb = R[i].finalBytes;
        if (p >= fb)
            continue;
        const uint32_t y = C[(size_t)i * m + i];
        uint4 x = gf_mul16(ld16(R[i].buf + p), c_inv[y]);
        x = mask16(x, (int)bb - (int)p); // zero beyond the recovered length
        st16(R[i].buf + p, x);
        if (p >= bb)
            continue;
        for (uint32_t j = 0; j < (uint32_t)i; ++j) {
            const uint32_t c = C[(size_t)j * m + i];
            if (!c)
                continue;
            const uint32_t ab = bb < R[j].finalBytes ? bb : R[j].finalBytes;
            if (p >= ab)
                continue;
            const uint4 xs = mask16(x, (int)ab - (int)p);
            st16(R[j].buf + p, xor16(ld16(R[j].buf + p), gf_mul16(xs, c)));
        }
    }
}

// ---------------------------------------------------------------------------
// Host side

namespace {

hipStream_t g_stream = nullptr;
bool g_ready = false;
bool g_timing = false;
double g_execMs = 0, g_totalMs = 0;

struct EvPair
{
    hipEvent_t a, b;
    bool exec;
};
std::vector<EvPair> g_evFree, g_evUsed;

EvPair take_events(bool exec)
{
    EvPair e;
    if (!g_evFree.empty()) {
        e = g_evFree.back();
        g_evFree.pop_back();
    } else {
        hipEventCreate(&e.a);
        hipEventCreate(&e.b);
    }
    e.exec = exec;
    return e;
}

struct Timed
{
    EvPair ev;
    bool on;
    explicit Timed(bool exec) : on(g_timing)
    {
        if (on) {
            ev = take_events(exec);
            hipEventRecord(ev.a, g_stream);
        }
    }
    ~Timed()
    {
        if (on) {
            hipEventRecord(ev.b, g_stream);
            g_evUsed.push_back(ev);
        }
    }
};

void check(hipError_t e, const char* what)
{
    if (e != hipSuccess) {
        std::fprintf(stderr, "siamese_amd: %s failed: %s\n", what, hipGetErrorString(e));
    }
}

} // namespace

bool be_init(int device, const char** err)
{
    if (g_ready)
        return true;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        *err = "no HIP device visible: libsiamese_amd requires an MI355X (gfx950)";
        return false;
    }
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        *err = "hipSetDevice failed";
        return false;
    }
    int cur = 0;
    hipGetDevice(&cur);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cur) != hipSuccess) {
        *err = "hipGetDeviceProperties failed";
        return false;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        *err = "device is not gfx950 (MI355X); kernels are built for gfx950 only";
        return false;
    }
    if (hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess) {
        *err = "hipStreamCreate failed";
        return false;
    }
    if (!gf_init()) {
        *err = "GF(256) table self-check failed";
        return false;
    }
    static uint32_t perm[256][8];
    for (unsigned y = 0; y < 256; ++y) {
        uint8_t ta[8], tb[8], tc[4];
        for (unsigned k = 0; k < 8; ++k) {
            ta[k] = gf_mul((uint8_t)k, (uint8_t)y);
            tb[k] = gf_mul((uint8_t)(k << 3), (uint8_t)y);
        }
        for (unsigned k = 0; k < 4; ++k)
            tc[k] = gf_mul((uint8_t)(k << 6), (uint8_t)y);
        std::memset(perm[y], 0, sizeof(perm[y]));
        std::memcpy(&perm[y][0], ta, 8);
        std::memcpy(&perm[y][2], tb, 8);
        std::memcpy(&perm[y][4], tc, 4);
    }
    check(hipMemcpyToSymbol(HIP_SYMBOL(c_perm), perm, sizeof(perm)), "hipMemcpyToSymbol(perm)");
    check(hipMemcpyToSymbol(HIP_SYMBOL(c_inv), g_gf.inv, 256), "hipMemcpyToSymbol(inv)");
    if (hipDeviceSynchronize() != hipSuccess) {
        *err = "device synchronisation failed during init";
        return false;
    }
    g_ready = true;
    return true;
}

const char* be_name() { return "hip-gfx950"; }

void* be_dev_alloc(size_t bytes)
{
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess)
        return nullptr;
    return p;
}

void be_dev_free(void* p)
{
    if (p)
        hipFree(p);
}

void* be_host_alloc(size_t bytes)
{
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess)
        return nullptr;
    return p;
}

void be_host_free(void* p)
{
    if (p)
        hipHostFree(p);
}

void be_h2d(void* dst, const void* src, size_t bytes)
{
    check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, g_stream), "H2D");
}

void be_d2h(void* dst, const void* src, size_t bytes)
{
    check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, g_stream), "D2H");
}

void be_memset(void* dst, int value, size_t bytes)
{
    check(hipMemsetAsync(dst, value, bytes, g_stream), "memset");
}

void be_launch_ingest(const IngestDesc* descs, const IngestItem* items, uint32_t count)
{
    Timed t(false);
    hipLaunchKernelGGL(k_ingest, dim3(count), dim3(64), 0, g_stream, descs, items);
}

void be_launch_exec(const GfOp* ops, const GfTerm* terms, const ExecItem* items, uint32_t count)
{
    Timed t(true);
    hipLaunchKernelGGL(k_exec, dim3(count), dim3(64), 0, g_stream, ops, terms, items);
}

void be_launch_solve_prefix(const SolveDesc* solves, const SolveRow* rows, const uint8_t* coef,
                            uint32_t* results, uint32_t count)
{
    Timed t(false);
    hipLaunchKernelGGL(k_solve_prefix, dim3(count), dim3(64), 0, g_stream, solves, rows, coef,
                       results);
}

void be_launch_solve_main(const SolveDesc* solves, const SolveRow* rows, const uint8_t* coef,
                          const uint32_t* results, const SolveItem* items, uint32_t count)
{
    Timed t(false);
    hipLaunchKernelGGL(k_solve_main, dim3(count), dim3(64), 0, g_stream, solves, rows, coef,
                       results, items);
}

bool be_sync()
{
    const hipError_t e = hipStreamSynchronize(g_stream);
    if (e != hipSuccess) {
        check(e, "hipStreamSynchronize");
        return false;
    }
    for (const EvPair& ev : g_evUsed) {
        float ms = 0;
        hipEventElapsedTime(&ms, ev.a, ev.b);
        g_totalMs += ms;
        if (ev.exec)
            g_execMs += ms;
        g_evFree.push_back(ev);
    }
    g_evUsed.clear();
    return true;
}

void be_timing_enable(bool on) { g_timing = on; }
void be_timing_reset()
{
    g_execMs = 0;
    g_totalMs = 0;
}
double be_timing_exec_ms() { return g_execMs; }
double be_timing_total_ms() { return g_totalMs; }

} // namespace sgpu
