// tools/backend_null.cpp -- PROFILING AID ONLY (never shipped, never tested
// against).  A backend.h implementation whose launches do no symbol work, so
// a bench run on the CPU measures the host control plane alone: stepping
// codecs, flush assembly and completions.
//
// The control plane only reads one thing back from the device: the
// recovered length words of each solve.  Here every solve reports all m rows
// valid with a 2-byte prefix and NULLSIM_LEN payload bytes (default 1400), so
// fixed-size workloads (C4, C2, C3) take the same control flow as on the GPU.
// Symbol bytes are garbage: run bench.py with verification off
// (--no-verify is implied by the digest-free timed steps).
#include "../siamese_amd/csrc/backend.h"
#include "../siamese_amd/csrc/gf.h"

#include <cstdlib>
#include <cstring>

namespace sgpu {

namespace {

// the last upload: device range -> host source (launch arguments point into it)
const uint8_t* g_upHost = nullptr;
uint8_t* g_upDev = nullptr;
size_t g_upBytes = 0;
uint32_t g_len = 1400;

template <class T>
const T* host_view(const T* dev)
{
    const uint8_t* p = reinterpret_cast<const uint8_t*>(dev);
    if (p >= g_upDev && p < g_upDev + g_upBytes)
        return reinterpret_cast<const T*>(g_upHost + (p - g_upDev));
    return dev;
}

} // namespace

bool be_init(int, const char** err)
{
    if (!gf_init()) {
        *err = "gf_init failed";
        return false;
    }
    if (const char* s = std::getenv("NULLSIM_LEN"))
        g_len = (uint32_t)std::strtoul(s, nullptr, 10);
    return true;
}

const char* be_name() { return "null (profiling only)"; }

void* be_dev_alloc(size_t bytes)
{
    void* p = nullptr;
    if (posix_memalign(&p, 256, bytes) != 0)
        return nullptr;
    return p;
}
void be_dev_free(void* p) { std::free(p); }
void* be_host_alloc(size_t bytes) { return be_dev_alloc(bytes); }
void* be_host_alloc_mapped(size_t bytes) { return be_dev_alloc(bytes); }
void be_host_free(void* p) { std::free(p); }
void* be_host_device_ptr(void*) { return nullptr; }   // (no zero-copy: uploads stay DMA-shaped)
void be_h2d(void* dst, const void* src, size_t bytes)
{
    // a DMA on the GPU: remember the mapping instead of copying
    g_upDev = (uint8_t*)dst;
    g_upHost = (const uint8_t*)src;
    g_upBytes = bytes;
}
void be_d2h(void* dst, const void* src, size_t bytes) { std::memcpy(dst, src, bytes); }
void be_copy_pinned(const BeCopy* r, unsigned n, bool toDevice)
{
    for (unsigned i = 0; i < n; ++i) {
        if (toDevice)
            be_h2d((void*)(uintptr_t)r[i].dst, (const void*)(uintptr_t)r[i].src, r[i].bytes);
        else
            be_d2h((void*)(uintptr_t)r[i].dst, (const void*)(uintptr_t)r[i].src, r[i].bytes);
    }
}
void be_copy_list(const BeCopy* r, const void*, unsigned n, bool toDevice) { be_copy_pinned(r, n, toDevice); }
void be_memset(void* dst, int value, size_t bytes) { std::memset(dst, value, bytes); }

void be_launch_ingest(const IngestDesc*, uint32_t, uint32_t, const uint32_t*, uint32_t) {}
void be_launch_exec(const void*, const ExecItem*, uint32_t, uint64_t*, const uint32_t*, uint32_t) {}
void be_launch_ldpc(const LdpcItem*, uint32_t, uint64_t*) {}

static void solve_prefix(const SolveDesc* solves, const SolveRow*, const uint8_t*,
                            uint32_t* results, uint32_t count, uint64_t*)
{
    const SolveDesc* sd = host_view(solves);
    for (uint32_t s = 0; s < count; ++s) {
        uint32_t* out = results + sd[s].result;
        out[0] = sd[s].m;
        for (uint32_t i = 0; i < sd[s].m; ++i)
            out[1 + i] = (2u << 29) | g_len;
    }
}

static void solve_main(const SolveDesc*, const SolveRow*, const uint8_t*, const uint32_t*,
                          const SolveItem*, uint32_t, uint32_t)
{
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
    (void)count;
    std::memcpy(hostOut, devStage, bytes);
    return true;
}

bool be_sync() { return true; }
void* be_fence() { return reinterpret_cast<void*>(1); }
bool be_fence_wait(void*, unsigned, bool) { return true; }
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
    const SolveItem* it = host_view(items);
    for (uint32_t k = 0; k < count; ++k)
        if (it[k].tileBase == 0)
            solve_prefix(solves + it[k].solve, rows, coef, results, 1, acct);
    solve_main(solves, rows, coef, results, items, count, maxRows);
}

// matrix jobs: every one reports an eliminated matrix with identity pivots,
// its first `cols` rows used and zero coefficients (no elimination on the host)
void be_side_upload_ingest(const BeCopy* rest, const IngestDesc*, uint32_t, uint32_t, const uint32_t*, uint32_t)
{
    if (rest)
        be_copy_pinned(rest, 1, true);
}

void be_launch_ge(const GeDesc* descs, const uint8_t*, uint32_t count, uint32_t* results, SolveRow*, uint8_t*,
                  uint32_t, uint32_t, const BeCopy* head, bool, const SolveRow*)
{
    if (head)
        be_copy_pinned(head, 1, true);
    const GeDesc* dd = host_view(descs);
    for (uint32_t j = 0; j < count; ++j) {
        const GeDesc d = dd[j];
        uint32_t* out = results + d.result;
        const bool chained = (d.flags & kGeChained) != 0;
        std::memset(out, 0, (size_t)ge_result_words(d.rows, d.cols, chained) * 4);
        out[0] = d.cols;
        out[3] = 1;
        uint8_t* po = reinterpret_cast<uint8_t*>(out + ge_out_pivots(d.rows));
        if (chained) {
            for (unsigned i = 0; i < d.rows; ++i)
                po[i] = (uint8_t)i;
            continue;
        }
        uint8_t* uo = reinterpret_cast<uint8_t*>(out + ge_out_used(d.rows));
        uint16_t* co = reinterpret_cast<uint16_t*>(out + ge_out_counts(d.rows));
        for (unsigned i = 0; i < d.rows; ++i) {
            po[i] = (uint8_t)i;
            uo[i] = i < d.cols;
            co[i] = (uint16_t)d.cols;
        }
    }
}

// (synchronous here)
void be_join_ge() {}

} // namespace sgpu
