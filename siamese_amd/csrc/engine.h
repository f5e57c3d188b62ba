// engine.h -- device-side resources of the codec: an arena of symbol
// buffers in HBM, per-instance op programs, and the flush that turns all
// pending programs into a handful of kernel launches.
#pragma once

#include "ops.h"

#include <cstdint>
#include <functional>
#include <mutex>
#include <vector>

namespace sgpu {

/// A symbol-sized buffer in device memory.  Capacity is a multiple of 64 B.
struct DevBuf
{
    uint8_t* ptr = nullptr;
    uint32_t cap = 0;
    explicit operator bool() const { return ptr != nullptr; }
    uint64_t addr() const { return (uint64_t)(uintptr_t)ptr; }
};

class Engine;

/// Ops of one codec instance since the last flush.  Segments are separated
/// by triangular solves; `group` orders instances inside a flush (group 0 =
/// encoders, which may feed group 1 = decoders).
class Program
{
public:
    Program(Engine* e, int group) : eng_(e), group_(group) {}
    ~Program();
    Program(const Program&) = delete;
    Program& operator=(const Program&) = delete;

    int group() const { return group_; }

    /// LINCOMB: dst[i] = (i < valid ? dst[i] : 0) ^ acc0 ^ mix*acc1, i < n.
    void lc_begin(uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix = 0);
    void lc_term(uint64_t src, uint32_t len, uint8_t coeff, uint8_t acc = 0);
    void lc_end();

    /// Convenience single-term forms of the reference bulk ops
    /// (reference gf256.h:249-266).
    void add_mem(uint64_t dst, uint64_t src, uint32_t n);             // dst ^= src
    void muladd_mem(uint64_t dst, uint8_t y, uint64_t src, uint32_t n);// dst ^= y*src
    void mul_mem(uint64_t dst, uint64_t src, uint8_t y, uint32_t n);   // dst = y*src
    void zero(uint64_t dst, uint32_t n);

    /// Writes <= 8 literal bytes at dst + offset.
    void literal(uint64_t dst, uint32_t offset, const uint8_t* bytes, uint32_t len);

    /// Ingest a symbol into a fresh buffer: dst = hdr || data.
    void ingest_host(const DevBuf& dst, const void* data, uint32_t bytes, const uint8_t* hdr,
                     uint32_t hdrLen);
    void ingest_device(const DevBuf& dst, uint64_t src, uint32_t bytes, const uint8_t* hdr,
                       uint32_t hdrLen);

    /// Queue a triangular solve; returns the result-word index it will fill
    /// (valid in the completion callback of the flush that runs it).
    uint32_t solve(const std::vector<SolveRow>& rows, const std::vector<uint8_t>& coef,
                   uint32_t maxBytes);

    bool empty() const { return segs_.empty() || (segs_.size() == 1 && segs_[0].ops.empty()); }

private:
    friend class Engine;
    struct Segment
    {
        std::vector<GfOp> ops;
        std::vector<GfTerm> terms;
        uint32_t maxExtent = 0;
    };
    struct PendingSolve
    {
        SolveDesc desc;
        std::vector<SolveRow> rows;
        std::vector<uint8_t> coef;
    };

    Segment& seg();
    void touch();

    Engine* eng_;
    int group_;
    bool dirty_ = false;
    bool open_ = false;       // inside lc_begin/lc_end
    std::vector<Segment> segs_;
    std::vector<PendingSolve> solves_;   // solve k follows segment k
};

class Engine
{
public:
    /// Process-wide engine used by the drop-in siamese.h entry points.
    static Engine* global();

    bool init(int device, const char** err);
    bool ready() const { return ready_; }

    DevBuf alloc(uint32_t bytes);
    void release(DevBuf& b);               // recycled after the next sync
    uint64_t bytes_in_use() const { return inUse_; }

    /// Copy `bytes` of device memory to host memory once the next flush has
    /// executed; the data is in place after sync().
    void download(void* hostDst, uint64_t devSrc, uint32_t bytes);

    /// Run `fn(results)` after the next flush completes; `results` is the
    /// solve-result word array of that flush.
    void on_complete(std::function<void(const uint32_t*)> fn);

    void flush();
    bool sync();
    bool flush_and_sync()
    {
        flush();
        return sync();
    }

    bool pending() const { return !dirty_.empty() || !ingest_.empty() || !downloads_.empty(); }

    /// Copy device ranges into one host buffer right now (after completing
    /// any flush in flight).  Queued, unflushed work is not touched.
    bool gather(unsigned count, const void* const* srcs, const unsigned* bytes, void* hostOut);

    std::mutex& mutex() { return mu_; }

    // statistics of the last flushes (for the bench / profiles)
    struct Stats
    {
        uint64_t flushes = 0, launches = 0, ops = 0, terms = 0, solves = 0, ingests = 0;
        uint64_t uploadBytes = 0;
        // Algorithmic bytes: source bytes of every bulk GF op
        // the reference codec performs for the same call sequence, and bytes
        // of recovery packets / recovered originals produced.
        uint64_t refOpBytes = 0, outBytes = 0;
        uint64_t solveBytes = 0;   // the part of both done by the solve kernels
    } stats;

    void account(uint64_t opBytes, uint64_t outBytes = 0, bool inSolve = false)
    {
        stats.refOpBytes += opBytes;
        stats.outBytes += outBytes;
        if (inSolve)
            stats.solveBytes += opBytes + outBytes;
    }

private:
    friend class Program;
    void register_dirty(Program* p) { dirty_.push_back(p); }
    void forget(Program* p);
    uint32_t reserve_results(uint32_t words)
    {
        const uint32_t r = resultWords_;
        resultWords_ += words;
        return r;
    }
    void stage_host_ingest(const DevBuf& dst, const void* data, uint32_t bytes, const uint8_t* hdr,
                           uint32_t hdrLen);
    void add_ingest(const IngestDesc& d, uint32_t hostStageOffset);

    bool ready_ = false;
    std::mutex mu_;

    // ---- arena ----
    struct Chunk
    {
        uint8_t* base;
        size_t size, used;
    };
    std::vector<Chunk> chunks_;
    std::vector<std::pair<uint32_t, std::vector<uint8_t*>>> freeLists_; // sorted by cap
    std::vector<DevBuf> pendingFree_;   // released since the last flush
    std::vector<DevBuf> flightFree_;    // released before the flush in flight
    uint64_t inUse_ = 0;
    std::vector<uint8_t*>* free_list(uint32_t cap);

    // ---- pending work ----
    std::vector<Program*> dirty_;
    struct IngestRec
    {
        IngestDesc d;
        int64_t hostOffset;   // >= 0: src lives in the host staging area
    };
    std::vector<IngestRec> ingest_;
    std::vector<uint8_t> hostStage_;   // host payloads awaiting H2D
    struct Download
    {
        void* host;
        uint64_t dev;
        uint32_t bytes;
    };
    std::vector<Download> downloads_;
    std::vector<std::function<void(const uint32_t*)>> callbacks_;
    uint32_t resultWords_ = 0;

    // ---- in flight ----
    struct InFlight
    {
        std::vector<Download> downloads;
        std::vector<std::function<void(const uint32_t*)>> callbacks;
        uint32_t resultWords = 0;
        size_t downloadBytes = 0;
        bool active = false;
    } flight_;

    // transfer buffers (grown on demand)
    uint8_t* upHost_ = nullptr;
    uint8_t* upDev_ = nullptr;
    size_t upCap_ = 0;
    uint8_t* downHost_ = nullptr;
    uint8_t* downDev_ = nullptr;   // device-side gather area for downloads + results
    size_t downCap_ = 0;
    void ensure_up(size_t bytes);
    void ensure_down(size_t bytes);

    // gather buffers (separate from the flush buffers)
    uint8_t* gUpHost_ = nullptr;
    uint8_t* gUpDev_ = nullptr;
    size_t gUpCap_ = 0;
    uint8_t* gHost_ = nullptr;
    uint8_t* gDev_ = nullptr;
    size_t gCap_ = 0;
};

} // namespace sgpu
