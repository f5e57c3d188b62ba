// tools/variants/solve_mfma.hip -- a MEASURED DEAD END, kept for the record;
// not built into libsiamese_amd.so.
//
// The decoder's bulk solve X = T R (T = U^-1 L^-1) on the int8 matrix cores:
// over GF(2) a GF(256) product is an 8x8 bit matrix, so X's bits are one
// binary matrix product, an integer dot product of 0/1 bytes whose low bit is
// the GF(2) sum (v_mfma_i32_32x32x32_i8).  Bit-exact on the GPU parity suite
// in round 4, but k_solve_pre 80 + k_solve_mfma 322 us per headline launch
// against 80 + 103 for the same product on the vector ALUs (k_solve_tr, the
// product path the library keeps): the matrix cores were busy 10 % of the
// kernel, the rest waited on LDS (profiles/r4k_pmc_summary.txt,
// r4l_kernel_stats.csv).  It used the product path's T (k_solve_pre) and the
// tile pass's copy of its scratch rows (k_solve_main flag bit 1); to revive it,
// paste it back after solve_tbuild with c_aff[256][8] (the GF2P8AFFINEQB bit
// matrices, filled by hipMemcpyToSymbol at init) and the group constants:
//   kMfmaTiles = 2, kMfmaChunk = 64, kMfmaGroupRows = 32,
//   kMfmaGroups = ceil(kProductMaxRows / 32),
//   LDS = 32*8*rows + rows*8*64 + 32*64 + align16(12 m) + 8 m + 16 bytes.

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(kMfmaThreads) void k_solve_mfma(const SolveDesc* __restrict__ solves,
                                                           const SolveRow* __restrict__ rows,
                                                           uint32_t* results)
{
    extern __shared__ uint4 Ls[];
    const uint32_t grp = blockIdx.x % kMfmaGroups;
    const SolveDesc sd = solves[blockIdx.x / kMfmaGroups];
    const uint32_t m = sd.m, mp = mfma_rows(m);
    if (m == 0 || m > kMfmaMaxRows || sd.tinv == 0 || grp * kMfmaGroupRows >= mp || results[sd.result] != m)
        return;   // (uniform: k_solve_main solves it, or another group has these rows)
    const SolveRow* R = rows + sd.rowBegin;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t row0 = grp * kMfmaGroupRows;

    uint8_t* AF = reinterpret_cast<uint8_t*>(Ls);                // [il][q][j]: c_aff[T[row0+il][j]][q]
    uint8_t* bits = AF + kMfmaGroupRows * 8u * mp;
    uint8_t* outT = bits + mp * 8u * kMfmaChunk;
    uint32_t* initB = reinterpret_cast<uint32_t*>(outT + kMfmaGroupRows * kMfmaChunk);
    uint32_t* finB = initB + m;
    uint32_t* bbB = finB + m;                                    // recovered header + length
    uint64_t* rowBuf = reinterpret_cast<uint64_t*>(bbB + ((m + 1u) & ~1u));

    const GMEM uint8_t* T = reinterpret_cast<const GMEM uint8_t*>(sd.tinv);
    for (uint32_t x = tid; x < kMfmaGroupRows * mp; x += kMfmaThreads) {
        const uint32_t il = x / mp, j = x - il * mp;
        const uint32_t i = row0 + il;
        const uint32_t y = (i < m && j < m) ? T[i * kMfmaYStride + j] : 0u;
        const uint2 a = *reinterpret_cast<const uint2*>(c_aff[y]);
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q)
            AF[(il * 8u + q) * mp + j] = (uint8_t)((q < 4 ? a.x : a.y) >> (8 * (q & 3)));
    }
    for (uint32_t j = tid; j < m; j += kMfmaThreads) {
        initB[j] = R[j].initBytes;
        finB[j] = R[j].finalBytes;
        rowBuf[j] = R[j].buf;
        const uint32_t w = results[sd.result + 1 + j];
        bbB[j] = (w >> 29) + (w & kSolveLengthMask);
    }
    __syncthreads();

    const uint32_t S = mp / 4;   // K steps (four input rows = 32 input bits each)
    uint32_t maxB = 0;
    for (uint32_t j = 0; j < m; ++j)
        maxB = finB[j] > maxB ? finB[j] : maxB;
    const uint32_t r = lane & 31, h = lane >> 5;
    // lane's A row: output bit 7 - (r & 7) of row row0 + 4 wave + r / 8
    const uint8_t* af = AF + ((4u * wave + (r >> 3)) * 8u + (7u - (r & 7u))) * mp + 2u * h;
    const bool active = row0 + 4u * wave < mp;
    const uint32_t rowsHere = (m - row0 < kMfmaGroupRows ? m - row0 : kMfmaGroupRows);
    const uint32_t xs = solve_x_stride(sd.maxBytes);
    for (uint32_t c0 = 0; c0 < maxB; c0 += kMfmaChunk) {
        // the B operand: byte (j, col) as eight 0/1 bytes at
        // bits[((t * S + j / 4) * 64 + (j % 4) / 2 * 32 + col % 32) * 16 + (j % 2) * 8],
        // t = col / 32 (lane h * 32 + r's 16-byte fragment of K step s is
        // contiguous, lanes in order: conflict-free ds_read_b128); item `it`
        // is the 8-byte slot it * 8, so a wave's stores are one contiguous
        // 512-byte run (the per-dword stores they replace were 16-way bank
        // conflicts: SQ_LDS_BANK_CONFLICT 47.7 M cycles per launch)
        for (uint32_t it = tid; it < mp * kMfmaChunk; it += kMfmaThreads) {
            const uint32_t blk = it >> 7, w = it & 127u;
            const uint32_t t = blk / S, g = blk - t * S;
            const uint32_t j = 4u * g + 2u * (w >> 6) + (w & 1u), col = 32u * t + ((w >> 1) & 31u);
            uint32_t v = 0;
            if (j < m) {
                const uint32_t p = c0 + col;
                if (p < initB[j])
                    v = *reinterpret_cast<const GMEM uint8_t*>(rowBuf[j] + p);
            }
            *reinterpret_cast<uint2*>(bits + 8u * it) = make_uint2(bits4(v), bits4(v >> 4));
        }
        __syncthreads();
        if (active) {
            i32x16 acc[kMfmaTiles];
#pragma unroll
            for (uint32_t t = 0; t < kMfmaTiles; ++t)
                acc[t] = i32x16{};
            for (uint32_t s = 0; s < S; ++s) {
                // A[r][16 h + jj]: bit b of T[i][4 s + 2 h + jj / 8] * 2^(jj % 8)
                const uint32_t u = *reinterpret_cast<const uint16_t*>(af + 4u * s);
                const i32x4 A = {(int)bits4(u), (int)bits4(u >> 4), (int)bits4(u >> 8), (int)bits4(u >> 12)};
#pragma unroll
                for (uint32_t t = 0; t < kMfmaTiles; ++t) {
                    const i32x4 B = *reinterpret_cast<const i32x4*>(bits + ((t * S + s) * 64 + h * 32 + r) * 16);
                    acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, acc[t], 0, 0, 0);
                }
            }
            // D[row][col]: row = (reg & 3) + 8 (reg >> 2) + 4 h, col = r; row
            // 8 g + 4 h + q is bit 4 h + q of output row 4 wave + g (local)
#pragma unroll
            for (uint32_t t = 0; t < kMfmaTiles; ++t)
#pragma unroll
                for (uint32_t g = 0; g < 4; ++g) {
                    const uint32_t nib = (acc[t][4 * g] & 1) | (acc[t][4 * g + 1] & 1) << 1 |
                                         (acc[t][4 * g + 2] & 1) << 2 | (acc[t][4 * g + 3] & 1) << 3;
                    const uint32_t v = nib << (4 * h);
                    const uint32_t byte = v | (uint32_t)__shfl_xor((int)v, 32);
                    if (h == 0)
                        outT[(4 * wave + g) * kMfmaChunk + t * 32 + r] = (uint8_t)byte;
                }
        }
        __syncthreads();
        // x masked past the recovered length, stored below the row's final
        // bytes (the stores of the exact back-substitution) into the result
        // scratch: another group may still read these rows' bytes; the tile
        // pass (k_solve_main) copies them into the rows
        // (a non-zero byte past a row's recovered length flags the solve for
        // the exact sweeps, as in k_solve_tr)
        uint32_t tail = 0;
        for (uint32_t it = tid; it < rowsHere * (kMfmaChunk / 16); it += kMfmaThreads) {
            const uint32_t il = it / (kMfmaChunk / 16), u = it % (kMfmaChunk / 16);
            const uint32_t i = row0 + il, p = c0 + 16 * u;
            const uint4 v = *reinterpret_cast<const uint4*>(outT + il * kMfmaChunk + 16 * u);
            const uint4 k = mask16(v, (int)bbB[i] - (int)p);
            tail |= (v.x ^ k.x) | (v.y ^ k.y) | (v.z ^ k.z) | (v.w ^ k.w);
            if (p < finB[i])
                st16(sd.xout + (uint64_t)i * xs + p, k);
        }
        if (__any(tail != 0) && lane == 0)
            atomicOr(results + sd.result + 1 + m, 1u);
    }
}


// Layout check of the int8 MFMA (tests): D = A B for 32 x 32 x 32 with
// asymmetric integer data, fragments as k_solve_mfma reads them.
__global__ void k_mfma_i8_check(int* __restrict__ out)
{
    const uint32_t l = threadIdx.x, r = l & 31, h = l >> 5;
    i32x4 A, B;
    int8_t* a = reinterpret_cast<int8_t*>(&A);
    int8_t* b = reinterpret_cast<int8_t*>(&B);
    for (uint32_t jj = 0; jj < 16; ++jj) {
        const uint32_t k = 16 * h + jj;
        a[jj] = (int8_t)((int)((r * 7 + k * 3) % 5) - 2);
        b[jj] = (int8_t)((int)((k * 11 + r * 5) % 7) - 3);
    }
    i32x16 acc = {};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, acc, 0, 0, 0);
    for (uint32_t reg = 0; reg < 16; ++reg) {
        const uint32_t row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        out[row * 32 + r] = acc[reg];
    }
}


// Test hook: the int8 MFMA fragment layout k_solve_mfma relies on, against
// the host's product of the same 32 x 32 x 32 integer matrices.  Returns the
// number of differing outputs (0: the layout holds), -1 on a device error.
extern "C" __attribute__((visibility("default"))) int sgpu_selftest_mfma_i8(void)
{
    bind_device();
    int* d = nullptr;
    if (hipMalloc(&d, 32 * 32 * sizeof(int)) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_mfma_i8_check, dim3(1), dim3(64), 0, g_stream, d);
    int h[32 * 32];
    const bool ok = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, g_stream) == hipSuccess &&
                    hipStreamSynchronize(g_stream) == hipSuccess;
    (void)hipFree(d);
    if (!ok)
        return -1;
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int want = 0;
            for (int k = 0; k < 32; ++k)
                want += ((i * 7 + k * 3) % 5 - 2) * ((k * 11 + j * 5) % 7 - 3);
            bad += h[i * 32 + j] != want;
        }
    return bad;
}
