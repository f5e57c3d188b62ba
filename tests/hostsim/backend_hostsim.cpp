// tests/hostsim/backend_hostsim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A CPU simulation of the backend.h contract, used solely by the CPU test
// suite to exercise the host control plane (encoder/decoder/engine) on a
// machine without a GPU.  It is linked into tests/hostsim/libsiamese_hostsim.so
// and NEVER into the product library siamese_amd/libsiamese_amd.so, whose
// only backend is backend_hip.hip.  The kernels' byte semantics are restated
// here one lane-tile at a time (including the v_perm_b32 GF(256) multiply),
// so a wrong op stream or table fails the same parity tests the GPU runs.
#include "../../siamese_amd/csrc/backend.h"
#include "../../siamese_amd/csrc/gf.h"
#include "../../siamese_amd/csrc/codedef.h"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace sgpu {

namespace {

uint32_t g_perm[256][8];
uint8_t g_inv[256];

// v_perm_b32 byte select for selector values 0..7 (and 12 -> 0)
uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel)
{
    const uint64_t data = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xff;
        uint32_t b = 0;
        if (s < 8)
            b = (uint32_t)(data >> (8 * s)) & 0xff;
        else if (s == 12)
            b = 0;
        else if (s >= 13)
            b = 0xff;
        r |= b << (8 * i);
    }
    return r;
}

uint32_t mul_dword(uint32_t x, uint32_t y)
{
    const uint32_t* t = g_perm[y];
    return perm(t[1], t[0], x & 0x07070707u) ^ perm(t[3], t[2], (x >> 3) & 0x07070707u) ^
           perm(0u, t[4], (x >> 6) & 0x03030303u);
}

void mul_bytes(uint8_t* v, unsigned n, uint8_t y)
{
    // operate dword-wise like the kernel
    for (unsigned i = 0; i < n; i += 4) {
        uint32_t w = 0;
        const unsigned k = n - i < 4 ? n - i : 4;
        std::memcpy(&w, v + i, k);
        w = mul_dword(w, y);
        std::memcpy(v + i, &w, k);
    }
}

int parse_prefix(const uint8_t* b, unsigned avail, unsigned* len)
{
    if (avail < 1)
        return -1;
    const unsigned top = b[0] >> 6;
    if (top <= 1) {
        *len = b[0];
        return 1;
    }
    if (top == 2) {
        if (avail < 2)
            return -1;
        *len = (((unsigned)b[0] << 8) | b[1]) & 0x3fff;
        return 2;
    }
    if ((b[0] & 0xE0) == 0xC0) {
        if (avail < 3)
            return -1;
        *len = (((unsigned)b[0] << 16) | ((unsigned)b[1] << 8) | b[2]) & 0x1fffff;
        return 3;
    }
    if (avail < 4)
        return -1;
    *len = (((unsigned)b[0] << 24) | ((unsigned)b[1] << 16) | ((unsigned)b[2] << 8) | b[3]) & 0x1fffffff;
    return 4;
}

inline uint8_t* P(uint64_t a) { return reinterpret_cast<uint8_t*>(a); }

// One linear combination on one tile: dst[0,n) = keep(dst,valid) ^ acc0 ^
// mix*acc1 with the terms (src, len, coeff, acc) given by `terms`.
struct TileTerm
{
    uint64_t src;
    uint32_t len;
    uint8_t coeff, acc;
    bool exact = false;   // read exactly len bytes (a clipped term), not through its last lane
};

void lincomb_tile(uint64_t dstAddr, uint32_t n, uint32_t valid, uint32_t mix,
                  const std::vector<TileTerm>& terms, uint32_t t0)
{
    const uint32_t t1 = t0 + kExecTileBytes;
    const uint32_t end = n < t1 ? n : t1;
    if (t0 >= end)
        return;
    const unsigned w = end - t0;
    uint8_t acc0[kExecTileBytes], acc1[kExecTileBytes], tmp[kExecTileBytes];
    std::memset(acc0, 0, w);
    std::memset(acc1, 0, w);
    for (const TileTerm& tm : terms) {
        if (t0 >= tm.len)
            continue;
        // read through the end of the term's last 16-byte lane, as the kernel
        // does: those bytes must be zero in memory (ops.h), and garbage there
        // shows up as a parity failure here
        const uint32_t lenA = tm.exact ? tm.len : (tm.len + 15) & ~15u;
        const unsigned k = (lenA < end ? lenA : end) - t0;
        std::memcpy(tmp, P(tm.src) + t0, k);
        if (tm.coeff != 1)
            mul_bytes(tmp, k, tm.coeff);
        uint8_t* acc = tm.acc ? acc1 : acc0;
        for (unsigned i = 0; i < k; ++i)
            acc[i] ^= tmp[i];
    }
    if (mix > 1)
        mul_bytes(acc1, w, (uint8_t)mix);
    uint8_t* dst = P(dstAddr) + t0;
    for (unsigned i = 0; i < w; ++i) {
        const uint8_t prior = (t0 + i < valid) ? dst[i] : 0;
        dst[i] = prior ^ acc0[i] ^ acc1[i];
    }
    // the kernel zero-fills the rest of the last 16-byte lane (ops.h)
    const uint32_t tailEnd = (n + 15) & ~15u;
    for (uint32_t b = n; b < tailEnd; ++b)
        if (b >= t0 && b < t1)
            P(dstAddr)[b] = 0;
}

void literal_tile(uint64_t dst, uint32_t at, const uint8_t* lit, uint32_t len, uint32_t t0)
{
    for (uint32_t k = 0; k < len; ++k) {
        const uint32_t b = at + k;
        if (b >= t0 && b < t0 + kExecTileBytes)
            P(dst)[b] = lit[k];
    }
}

void exec_tile(const uint8_t* stream, const ExecItem& it, uint32_t t0, uint64_t* acct, const uint32_t* results)
{
    const uint8_t* w = stream + (size_t)it.streamBegin * 16;
    const uint8_t* end = w + (size_t)it.streamWords * 16;
    std::vector<TileTerm> terms;
    for (uint32_t oi = 0; oi < it.opCount; ++oi) {
        GfOp op;
        std::memcpy(&op, w, sizeof(op));
        const uint8_t* body = w + sizeof(GfOp);
        w += (size_t)op_words(op) * 16;
        if (w > end)
            std::abort(); // malformed stream
        // (a gated op of a chained elimination that failed: termBegin, ops.h)
        if (op.kind != OP_LITERAL && op.termBegin != 0 && results[op.termBegin - 1] == 0)
            continue;
        if (op.kind == OP_LITERAL) {
            literal_tile(op.dst, op.n, op.lit, op.valid, t0);
            continue;
        }
        if (op.kind == OP_LINCOMB) {
            terms.clear();
            const GfTerm* tt = reinterpret_cast<const GfTerm*>(body);
            for (uint32_t k = 0; k < op.termCount; ++k)
                terms.push_back(TileTerm{tt[k].src, tt[k].len, tt[k].coeff, tt[k].acc});
            lincomb_tile(op.dst, op.n, op.valid, op.mix, terms, t0);
            continue;
        }
        if (op.kind == OP_LINCOMBS) {
            const LcItem* items = reinterpret_cast<const LcItem*>(body);
            const GfTerm* words = reinterpret_cast<const GfTerm*>(body);
            if (body + (size_t)op.termCount * 16 != w)
                std::abort(); // malformed block
            for (uint32_t i = 0; i < op.n; ++i) {
                const LcItem& it = items[i];
                if (it.termStart + it.termCount > op.termCount)
                    std::abort();
                terms.clear();
                for (uint32_t k = 0; k < it.termCount; ++k) {
                    const GfTerm& g = words[it.termStart + k];
                    terms.push_back(TileTerm{g.src, g.len, g.coeff, g.acc});
                }
                lincomb_tile(it.dst, it.n, it.valid, (uint8_t)(it.mixLit & 0xff), terms, t0);
                const uint32_t litLen = (it.mixLit >> 8) & 0xff;
                if (litLen)
                    literal_tile(it.dst, it.litOffset, it.lit, litLen, t0);
            }
            continue;
        }
        if (op.kind == OP_COPIES) {
            const CopyItem* cs = reinterpret_cast<const CopyItem*>(body);
            if (reinterpret_cast<const uint8_t*>(cs + op.n) != w)
                std::abort(); // malformed block
            for (uint32_t c = 0; c < op.n; ++c) {
                const uint32_t end16 = (cs[c].len + 15) & ~15u;
                for (uint32_t b = t0; b < t0 + kExecTileBytes && b < end16; ++b)
                    P(cs[c].dst)[b] = b < cs[c].len ? P(cs[c].src)[b] : 0;
            }
            continue;
        }
        if (op.kind != OP_ROWS)
            std::abort();
        // OP_ROWS (ops.h): sums, window, sum updates, rows
        const uint32_t E = op.valid, U = op.mix, R = op.n;
        const WinEntry* sums = reinterpret_cast<const WinEntry*>(body);
        const WinEntry* win = sums + kRowSums;
        const SumUpdate* ups = reinterpret_cast<const SumUpdate*>(win + E);
        const RowItem* rows = reinterpret_cast<const RowItem*>(ups + U);
        if (reinterpret_cast<const uint8_t*>(rows + R) != w)
            std::abort(); // malformed block
        for (uint32_t u = 0; u < U; ++u) {
            const SumUpdate& up = ups[u];
            terms.clear();
            for (uint32_t e = up.from; e < up.to; e += kLanes) {
                if (e >= E)
                    std::abort();
                const WinEntry& x = win[e];
                if (x.len == 0)
                    continue;
                uint8_t c = 1;
                if (up.s > 0) {
                    c = column_value(x.column);
                    if (up.s == 2)
                        c = gf_sqr(c);
                }
                terms.push_back(TileTerm{x.src, x.len, c, 0});
                if (t0 == 0)
                    *acct += x.len;   // the reference's source bytes (device-counted)
            }
            lincomb_tile(((uint64_t)up.dstHi << 32) | up.dstLo, up.n, up.valid, 0, terms, t0);
        }
        for (uint32_t r = 0; r < R; ++r) {
            const RowItem& h = rows[r];
            terms.clear();
            for (unsigned k = 0; k < kRowSums; ++k) {
                // (exactly the sum's first len bytes: an update of this batch
                // may have grown it past what the row reads, ops.h RowItem)
                if ((h.mask0 >> k & 1) && sums[k].len)
                    terms.push_back(TileTerm{sums[k].src, sums[k].len, 1, 0, true});
                if ((h.mask1 >> k & 1) && sums[k].len)
                    terms.push_back(TileTerm{sums[k].src, sums[k].len, 1, 1, true});
            }
            // versioned sum reads (ops.h RowItem.cutoff): take back out the
            // update elements at or past the row's cutoff
            for (uint32_t u = 0; u < U; ++u) {
                const SumUpdate& up = ups[u];
                const uint32_t k = up.sum;
                const bool in[2] = {(h.mask0 >> k & 1) != 0 && k < kRowSums, (h.mask1 >> k & 1) != 0 && k < kRowSums};
                if (!in[0] && !in[1])
                    continue;
                // (clipped to the sum's length as the row reads it)
                const uint32_t slen = sums[k].len;
                for (uint32_t e = up.from; e < up.to; e += kLanes) {
                    if (e < h.cutoff || win[e].len == 0)
                        continue;
                    uint8_t c = 1;
                    if (up.s > 0) {
                        c = column_value(win[e].column);
                        if (up.s == 2)
                            c = gf_sqr(c);
                    }
                    const uint32_t len = win[e].len < slen ? win[e].len : slen;
                    for (uint8_t a = 0; a < 2; ++a)
                        if (in[a] && len)
                            terms.push_back(TileTerm{win[e].src, len, c, a, len < win[e].len});
                }
            }
            if (h.mask0 & kRowWide) {
                // L0 / L1 of a wide row (k_ldpc), as two draws
                for (uint32_t i = 0; i < 2; ++i) {
                    const WinEntry& x = win[h.ldpcOff + i];
                    if (h.ldpcOff + i >= E)
                        std::abort();
                    terms.push_back(TileTerm{x.src, x.len, 1, (uint8_t)i});
                }
            }
            Pcg32 prng;
            prng.seed(h.row, h.ldpcN);
            const uint32_t pairs = (h.ldpcN + kPairRate - 1) / kPairRate;
            for (uint32_t i = 0; i < 2 * pairs; ++i) {
                const uint32_t e = h.ldpcOff + prng.next() % h.ldpcN;
                if (e >= E)
                    std::abort();
                if (win[e].len)
                    terms.push_back(TileTerm{win[e].src, win[e].len, 1, (uint8_t)(i & 1)});
                if (t0 == 0)
                    *acct += win[e].len < h.n ? win[e].len : h.n;
            }
            lincomb_tile(h.dst, h.n, h.valid, h.mask1 >> 24, terms, t0);
            literal_tile(h.dst, h.n, h.lit, row_lit_len(h.mask0), t0);
        }
    }
}

} // namespace

bool be_init(int, const char** err)
{
    if (!gf_init()) {
        *err = "gf_init failed";
        return false;
    }
    for (unsigned y = 0; y < 256; ++y) {
        uint8_t ta[8], tb[8], tc[4];
        for (unsigned k = 0; k < 8; ++k) {
            ta[k] = gf_mul((uint8_t)k, (uint8_t)y);
            tb[k] = gf_mul((uint8_t)(k << 3), (uint8_t)y);
        }
        for (unsigned k = 0; k < 4; ++k)
            tc[k] = gf_mul((uint8_t)(k << 6), (uint8_t)y);
        std::memset(g_perm[y], 0, sizeof(g_perm[y]));
        std::memcpy(&g_perm[y][0], ta, 8);
        std::memcpy(&g_perm[y][2], tb, 8);
        std::memcpy(&g_perm[y][4], tc, 4);
    }
    std::memcpy(g_inv, g_gf.inv, 256);
    return true;
}

const char* be_name() { return "hostsim (test only)"; }

void* be_dev_alloc(size_t bytes)
{
    void* p = nullptr;
    if (posix_memalign(&p, 256, bytes) != 0)
        return nullptr;
    std::memset(p, 0xA5, bytes); // garbage, like fresh device memory
    return p;
}
void be_dev_free(void* p) { std::free(p); }
void* be_host_alloc(size_t bytes) { return be_dev_alloc(bytes); }
void* be_host_alloc_mapped(size_t bytes) { return be_dev_alloc(bytes); }
void be_host_free(void* p) { std::free(p); }
void be_h2d(void* dst, const void* src, size_t bytes) { std::memcpy(dst, src, bytes); }
void* be_host_device_ptr(void* host) { return host; }
void be_d2h(void* dst, const void* src, size_t bytes) { std::memcpy(dst, src, bytes); }
void be_copy_pinned(const BeCopy* r, unsigned n, bool)
{
    for (unsigned i = 0; i < n; ++i)
        std::memcpy((void*)(uintptr_t)r[i].dst, (const void*)(uintptr_t)r[i].src, r[i].bytes);
}
void be_copy_list(const BeCopy* r, const void*, unsigned n, bool toDevice) { be_copy_pinned(r, n, toDevice); }
void be_memset(void* dst, int value, size_t bytes) { std::memset(dst, value, bytes); }

static bool noexec();

static void ingest_one(const IngestDesc& run, uint32_t k)
{
    IngestDesc d = run;
    d.dst2 = (d.dst2Mask >> k & 1u) ? d.dst2 + (uint64_t)k * d.dstStride : 0;
    d.src += (uint64_t)k * d.srcStride;
    d.dst += (uint64_t)k * d.dstStride;
    const uint32_t total = d.hdrLen + d.bytes;
    // the kernel stores whole 16-byte lanes, zero past the symbol
    const uint32_t end = (total + 15) & ~15u;
    for (uint32_t b = 0; b < end; ++b)
        P(d.dst)[b] = b < d.hdrLen ? d.hdr[b] : (b < total ? P(d.src)[b - d.hdrLen] : 0);
    if (d.dst2)
        std::memcpy(P(d.dst2), P(d.dst), end);
}

// The kernel's work assignment, block by block (a symbol the host's block
// table misses is not copied here either)
void be_launch_ingest(const IngestDesc* descs, uint32_t count, uint32_t, const uint32_t* blocks, uint32_t nblocks)
{
    if (noexec())
        return;
    if (!blocks) {
        for (uint32_t i = 0; i < count; ++i)
            ingest_one(descs[i], 0);
        return;
    }
    for (uint32_t b = 0; b < nblocks; ++b) {
        const uint32_t di = blocks[b] >> 4;
        if (di >= count)
            continue;
        const IngestDesc& d = descs[di];
        const uint32_t n = d.count ? d.count : 1u;
        for (uint32_t w = 0; w < kIngestWaves; ++w) {
            const uint32_t k = (blocks[b] & 15u) * kIngestWaves + w;
            if (k < n)
                ingest_one(d, k);
        }
    }
}

// HOSTSIM_NOEXEC=1 skips all symbol arithmetic so the host control plane
// can be timed on its own (profiling aid; results are fabricated lengths
// that are only valid for fixed-size 1400-byte payloads).
static bool noexec()
{
    static int v = -1;
    if (v < 0)
        v = std::getenv("HOSTSIM_NOEXEC") ? 1 : 0;
    return v == 1;
}

void be_launch_exec(const void* stream, const ExecItem* items, uint32_t count, uint64_t* acct,
                    const uint32_t* results, uint32_t)
{
    if (noexec())
        return;
    // (tile by tile: every op is local to its byte columns, so this order
    // gives the device's op-by-op, tile-by-tile results)
    for (uint32_t i = 0; i < count; ++i)
        for (uint32_t t = 0; t < exec_tile_count(items[i].tiles); ++t)
            exec_tile(static_cast<const uint8_t*>(stream), items[i],
                      (exec_first_tile(items[i].tiles) + t) * kExecTileBytes, acct, results);
}

void be_launch_ldpc(const LdpcItem* items, uint32_t count, uint64_t* acct)
{
    if (noexec())
        return;
    for (uint32_t k = 0; k < count; ++k) {
        const LdpcItem& it = items[k];
        const WinEntry* win = reinterpret_cast<const WinEntry*>((uintptr_t)it.win);
        Pcg32 prng;
        prng.seed(it.row, it.N);
        for (uint32_t d = 0; d < 2 * it.pair0; ++d)
            (void)prng.next();
        const uint32_t t1 = it.tileBase + kLdpcTileBytes;
        for (uint32_t d = 2 * it.pair0; d < 2 * it.pair1; ++d) {
            const WinEntry& x = win[it.off + prng.next() % it.N];
            if (it.tileBase == 0)
                *acct += x.len < it.n ? x.len : it.n;
            uint8_t* dst = P(it.dst + ((d & 1) ? it.span : 0));
            for (uint32_t b = it.tileBase; b < t1 && b < x.len; ++b)
                dst[b] ^= P(x.src)[b];
        }
    }
}

static void solve_prefix(const SolveDesc* solves, const SolveRow* rows, const uint8_t* coef,
                            uint32_t* results, uint32_t count, uint64_t* acct)
{
    for (uint32_t s = 0; s < count; ++s) {
        const SolveDesc& sd = solves[s];
        if (sd.gate && results[sd.gate - 1] == 0)
            continue;   // (a chained elimination that failed, ops.h GeDesc)
        const uint32_t m = sd.m;
        const SolveRow* R = rows + sd.rowBegin;
        const uint8_t* C = coef + sd.coefOffset;
        uint32_t* out = results + sd.result;
        if (noexec()) {
            out[0] = m;
            for (uint32_t i = 0; i < m; ++i)
                out[1 + i] = (2u << 29) | (R[i].finalBytes - 2);
            continue;
        }
        std::vector<uint8_t> pre((size_t)m * 4, 0);
        for (uint32_t j = 0; j < m; ++j)
            for (uint32_t b = 0; b < 4 && b < R[j].initBytes; ++b)
                pre[j * 4 + b] = P(R[j].buf)[b];
        for (uint32_t i = 0; i + 1 < m; ++i)
            for (uint32_t j = i + 1; j < m; ++j) {
                const uint8_t y = C[(size_t)j * m + i];
                if (!y)
                    continue;
                for (uint32_t b = 0; b < 4 && b < R[i].lowerLen; ++b)
                    pre[j * 4 + b] ^= gf_mul(pre[i * 4 + b], y);
            }
        uint32_t ok = 0;
        for (int i = (int)m - 1; i >= 0; --i) {
            const uint32_t fb = R[i].finalBytes;
            const uint32_t lc = fb < 32 ? fb : 32;
            const uint8_t inv = g_inv[C[(size_t)i * m + i]];
            uint8_t x[4] = {0, 0, 0, 0};
            for (uint32_t b = 0; b < 4 && b < lc; ++b)
                x[b] = gf_mul(pre[i * 4 + b], inv);
            unsigned len = 0;
            const int h = parse_prefix(x, lc, &len);
            if (h < 1 || len == 0 || (uint32_t)h + len > fb)
                break;
            out[1 + i] = ((uint32_t)h << 29) | len;
            const uint32_t bb = (uint32_t)h + len;
            ++ok;
            acct[0] += lc > bb ? lc : bb;
            acct[1] += bb;
            for (uint32_t j = 0; j < (uint32_t)i; ++j) {
                const uint8_t c = C[(size_t)j * m + i];
                if (!c)
                    continue;
                const uint32_t ab = bb < R[j].finalBytes ? bb : R[j].finalBytes;
                acct[0] += ab;
                for (uint32_t b = 0; b < 4 && b < ab; ++b)
                    pre[j * 4 + b] ^= gf_mul(x[b], c);
            }
        }
        out[0] = ok;
    }
}

static void solve_main(const SolveDesc* solves, const SolveRow* rows, const uint8_t* coef,
                          const uint32_t* results, const SolveItem* items, uint32_t count,
                          uint32_t)
{
    if (noexec())
        return;
    for (uint32_t it = 0; it < count; ++it) {
        const SolveDesc& sd = solves[items[it].solve];
        if (sd.gate && results[sd.gate - 1] == 0)
            continue;
        const uint32_t m = sd.m;
        const SolveRow* R = rows + sd.rowBegin;
        const uint8_t* C = coef + sd.coefOffset;
        const uint32_t* res = results + sd.result;
        const uint32_t t0 = items[it].tileBase, t1 = t0 + solve_tile_bytes(m);
        auto clip = [&](uint32_t v) { return v < t1 ? v : t1; };
        for (uint32_t j = 0; j < m; ++j)
            for (uint32_t b = (R[j].initBytes > t0 ? R[j].initBytes : t0); b < clip(R[j].finalBytes); ++b)
                P(R[j].buf)[b] = 0;
        for (uint32_t i = 0; i + 1 < m; ++i) {
            const uint32_t L = clip(R[i].lowerLen);
            if (t0 >= L)
                continue;
            for (uint32_t j = i + 1; j < m; ++j) {
                const uint8_t y = C[(size_t)j * m + i];
                if (!y)
                    continue;
                for (uint32_t b = t0; b < L; ++b)
                    P(R[j].buf)[b] ^= gf_mul(P(R[i].buf)[b], y);
            }
        }
        const uint32_t ok = res[0];
        for (int i = (int)m - 1; i >= 0; --i) {
            if ((uint32_t)(m - 1 - i) >= ok)
                break;
            const uint32_t w = res[1 + i];
            const uint32_t bb = (w >> 29) + (w & kSolveLengthMask);
            const uint32_t fb = clip(R[i].finalBytes);
            const uint8_t inv = g_inv[C[(size_t)i * m + i]];
            for (uint32_t b = t0; b < fb; ++b)
                P(R[i].buf)[b] = b < bb ? gf_mul(P(R[i].buf)[b], inv) : 0;
            // the kernel stores whole 16-byte lanes for every byte below the
            // row's final length, zero past the recovered length: bytes up to
            // align16(finalBytes) read as zero afterwards (a pending slot's
            // length bound is finalBytes, siamese_amd/csrc/decoder.h)
            const uint32_t fbEnd = (R[i].finalBytes > bb ? R[i].finalBytes : bb);
            for (uint32_t b = fb > t0 ? fb : t0; b < clip((fbEnd + 15) & ~15u); ++b)
                P(R[i].buf)[b] = 0;
            for (uint32_t j = 0; j < (uint32_t)i; ++j) {
                const uint8_t c = C[(size_t)j * m + i];
                if (!c)
                    continue;
                const uint32_t ab = clip(bb < R[j].finalBytes ? bb : R[j].finalBytes);
                for (uint32_t b = t0; b < ab; ++b)
                    P(R[j].buf)[b] ^= gf_mul(P(R[i].buf)[b], c);
            }
        }
    }
}

void* be_stage_h2d(void* dst, const void* src, size_t bytes)
{
    std::memcpy(dst, src, bytes);
    return reinterpret_cast<void*>(1);
}
void be_wait_mark(void*) {}
void be_mark_release(void*) {}
bool be_mark_sync(void*) { return true; }
// (synchronous here: both marks are passed on return)
bool be_gather(const IngestDesc* descsHost, void* descsDev, uint32_t count, const void* devStage,
               void* hostOut, size_t bytes, void** packed, void** landed)
{
    *packed = *landed = reinterpret_cast<void*>(1);
    std::memcpy(descsDev, descsHost, (size_t)count * sizeof(IngestDesc));
    be_launch_ingest(static_cast<const IngestDesc*>(descsDev), count, 0);
    std::memcpy(hostOut, devStage, bytes);
    return true;
}

// HOSTSIM_FAIL_SYNC=N: the N-th be_sync (1-based) and every later one
// report a device fault (tests of the sticky Disabled path).
bool be_sync()
{
    static std::atomic<long> failAt{-2};
    static std::atomic<long> calls{0};
    if (failAt == -2) {
        const char* v = std::getenv("HOSTSIM_FAIL_SYNC");
        failAt = v ? std::atol(v) : -1;
    }
    const long c = ++calls;
    return failAt < 1 || c < failAt;
}
// fences are synchronisations too (they count toward HOSTSIM_FAIL_SYNC)
void* be_fence() { return reinterpret_cast<void*>(1); }
bool be_fence_wait(void*, unsigned, bool) { return be_sync(); }
void be_timing_enable(bool) {}
void be_timing_reset() {}
double be_timing_kernel_ms(BeKernel) { return 0; }
double be_timing_exec_ms() { return 0; }
double be_timing_total_ms() { return 0; }


void be_launch_solve(const SolveDesc* solves, const SolveRow* rows, const uint8_t* coef, uint32_t* results,
                     const SolveItem* items, uint32_t count, uint32_t maxRows, uint64_t* acct,
                     uint32_t, uint32_t)
{
    // the device fuses both passes; here the prefix of each solve (its tile-0
    // item), then every tile
    for (uint32_t k = 0; k < count; ++k)
        if (items[k].tileBase == 0)
            solve_prefix(solves + items[k].solve, rows, coef, results, 1, acct);
    solve_main(solves, rows, coef, results, items, count, maxRows);
}

// k_ge: a fresh recovery matrix from its job (generation as the host's
// generate_matrix, reference SiameseDecoder.cpp:2157-2383), then the
// elimination without pivoting while the pivots allow it and with row
// pivoting from the first zero pivot (:2423-2531), as the kernel runs it.
void be_side_upload_ingest(const BeCopy* rest, const IngestDesc* descs, uint32_t count, uint32_t maxBytes,
                           const uint32_t* blocks, uint32_t nblocks)
{
    if (rest)
        be_copy_pinned(rest, 1, true);
    be_launch_ingest(descs, count, maxBytes, blocks, nblocks);
}

void be_launch_ge(const GeDesc* descs, const uint8_t* in, uint32_t count, uint32_t* results, SolveRow* srows,
                  uint8_t* scoef, uint32_t, uint32_t, const BeCopy* head, bool, const SolveRow* srowsIn)
{
    if (!srowsIn)
        srowsIn = srows;
    if (head)
        be_copy_pinned(head, 1, true);
    for (uint32_t jb = 0; jb < count; ++jb) {
        const GeDesc d = descs[jb];
        const unsigned rows = d.rows, cols = d.cols;
        const GeRow* R = reinterpret_cast<const GeRow*>(in + d.in);
        const GeCol* C = reinterpret_cast<const GeCol*>(R + rows);
        const uint8_t* pick = reinterpret_cast<const uint8_t*>(C + cols);
        std::vector<uint8_t> M((size_t)rows * cols, 0);
        for (unsigned r = 0; r < rows; ++r) {
            const GeRow& g = R[r];
            uint8_t* row = &M[(size_t)r * cols];
            const uint8_t rx = row_value(g.row);
            for (unsigned j = 0; j < g.jEnd && j < cols; ++j) {
                if (g.kind == GE_PARITY) {
                    row[j] = 1;
                } else if (g.kind == GE_CAUCHY) {
                    row[j] = gf_inv((uint8_t)(g.rbase ^ C[j].ccol));
                } else {
                    const unsigned op = row_opcode(C[j].lane, g.row);
                    auto comb = [&](unsigned k) {
                        return (uint8_t)((k & 1) ^ ((k & 2) ? C[j].cx : 0) ^ ((k & 4) ? C[j].cx2 : 0));
                    };
                    row[j] = (uint8_t)(comb(op & 7) ^ gf_mul(comb(op >> 3), rx));
                }
            }
            if (g.kind != GE_SIAMESE || g.ldpcN == 0)
                continue;
            Pcg32 prng;
            prng.seed(g.row, g.ldpcN);
            const unsigned picks = 2 * ((g.ldpcN + kPairRate - 1) / kPairRate);
            for (unsigned k = 0; k < picks; ++k) {
                const uint8_t c = pick[g.pickOff + prng.next() % g.ldpcN];
                if (c < cols)
                    row[c] ^= (k & 1) ? rx : 1;
            }
        }
        std::vector<uint8_t> piv(rows), used(rows, 0);
        std::vector<uint16_t> cnt(rows);
        for (unsigned i = 0; i < rows; ++i) {
            piv[i] = (uint8_t)i;
            cnt[i] = R[i].colCount;
        }
        uint64_t bytes = 0;
        auto elim = [&](unsigned src, unsigned dst, unsigned p, unsigned end, uint8_t val) {
            uint8_t* a = &M[(size_t)dst * cols];
            const uint8_t* b = &M[(size_t)src * cols];
            if (a[p] == 0)
                return false;
            const uint8_t y = gf_div(a[p], val);
            a[p] = y;
            if (end > p + 1) {
                for (unsigned c = p + 1; c < end; ++c)
                    a[c] ^= gf_mul(b[c], y);
                bytes += end - p - 1;
            }
            return true;
        };
        unsigned p = 0;
        for (; p < cols; ++p) {
            const uint8_t val = M[(size_t)p * cols + p];
            if (val == 0)
                break;
            used[p] = 1;
            for (unsigned k = p + 1; k < rows; ++k)
                elim(p, k, p, cnt[p], val);
        }
        unsigned stop = cols;
        if (p < cols) {
            unsigned j = p + 1;
            for (unsigned pivot = p; pivot < cols; ++pivot) {
                if (pivot != p)
                    j = pivot;
                while (j < rows && M[(size_t)piv[j] * cols + pivot] == 0)
                    ++j;
                if (j >= rows) {
                    stop = pivot;
                    break;
                }
                const unsigned rj = piv[j];
                std::swap(piv[pivot], piv[j]);
                used[rj] = 1;
                const unsigned end = cnt[rj];
                if (pivot >= cols - 1)
                    break;
                const uint8_t val = M[(size_t)rj * cols + pivot];
                for (unsigned k = pivot + 1; k < rows; ++k) {
                    const unsigned rk = piv[k];
                    if (elim(rj, rk, pivot, end, val) && cnt[rk] < end)
                        cnt[rk] = (uint16_t)end;
                }
            }
        }
        const bool ok = stop == cols;
        uint32_t nz = 0;   // non-zero multipliers below the diagonal, pivot order
        if (ok)
            for (unsigned j = 0; j < cols; ++j)
                for (unsigned i = 0; i < j; ++i)
                    nz += M[(size_t)piv[j] * cols + i] != 0;
        uint32_t* out = results + d.result;
        std::memset(out, 0, kGeOutHeader * 4);
        out[0] = stop;
        out[1] = (uint32_t)bytes;
        out[2] = (uint32_t)(bytes >> 32);
        out[3] = ok ? 1 : 0;
        out[4] = nz;
        uint8_t* po = reinterpret_cast<uint8_t*>(out + ge_out_pivots(rows));
        if (d.flags & kGeChained) {
            std::memset(po, 0, 4 * ((rows + 3) / 4));
            for (unsigned i = 0; i < rows; ++i)
                po[i] = piv[i];
            if (!ok)
                continue;
            uint8_t* co = scoef + d.solveCoef;
            for (unsigned j = 0; j < cols; ++j)
                std::memcpy(co + (size_t)j * cols, &M[(size_t)piv[j] * cols], cols);
            SolveRow* sr = srows + d.solveRow;
            std::vector<SolveRow> t(srowsIn + d.solveRow, srowsIn + d.solveRow + cols);
            for (unsigned j = 0; j < cols; ++j) {
                sr[j] = t[piv[j]];
                sr[j].headIndex = 1 + solve_head_slot(t[piv[j]].headIndex, piv[j]);
            }
            continue;
        }
        uint8_t* uo = reinterpret_cast<uint8_t*>(out + ge_out_used(rows));
        uint16_t* co = reinterpret_cast<uint16_t*>(out + ge_out_counts(rows));
        std::memset(po, 0, 4 * ((rows + 3) / 4));
        std::memset(uo, 0, 4 * ((rows + 3) / 4));
        std::memset(co, 0, 4 * ((rows + 1) / 2));
        for (unsigned i = 0; i < rows; ++i) {
            po[i] = piv[i];
            uo[i] = used[i];
            co[i] = cnt[i];
        }
        uint8_t* mo = reinterpret_cast<uint8_t*>(out + ge_out_matrix(rows));
        std::memset(mo, 0, 4 * ((rows * cols + 3) / 4));
        std::memcpy(mo, M.data(), M.size());
    }
}

// (synchronous here)
void be_join_ge() {}

} // namespace sgpu
