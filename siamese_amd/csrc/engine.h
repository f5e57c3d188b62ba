// engine.h -- device-side resources of the codec: an arena of symbol
// buffers in HBM, per-instance op programs, and the flush that turns all
// pending programs into a handful of kernel launches.
//
// Threading: codec instances may be driven concurrently from different host
// threads (one thread per instance at a time).  Everything an instance call
// touches in the engine lives in the calling thread's Shard (buffer free
// lists, ingest queue, downloads, statistics) or in the instance's own
// Program, so per-instance calls take no global lock.  flush()/sync()/
// gather() are exclusive: the caller guarantees no instance call runs
// concurrently with them (the siamese_gpu.h contract).
#pragma once

#include "ops.h"

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <vector>

namespace sgpu {

class WorkerPool;

/// A symbol-sized buffer in device memory.  Capacity is a multiple of 64 B.
struct DevBuf
{
    uint8_t* ptr = nullptr;
    uint32_t cap = 0;
    explicit operator bool() const { return ptr != nullptr; }
    uint64_t addr() const { return (uint64_t)(uintptr_t)ptr; }
};

class Engine;
struct Shard;

/// Completion callback of a flush; `results` is the solve-result word array
/// as seen by the program that registered it (indices returned by solve()).
using Completion = std::function<void(const uint32_t* results)>;

/// Ops of one codec instance since the last flush.  Segments are separated
/// by triangular solves; `group` orders instances inside a flush (group 0 =
/// encoders, which may feed group 1 = decoders).
class Program
{
public:
    Program(Engine* e, int group) : eng_(e), group_(group) { take_store(); }
    ~Program();
    Program(const Program&) = delete;
    Program& operator=(const Program&) = delete;

    int group() const { return group_; }

    /// LINCOMB: dst[i] = (i < valid ? dst[i] : 0) ^ acc0 ^ mix*acc1, i < n.
    void lc_begin(uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix = 0);
    // (lc_term must follow lc_begin directly: it appends to the last op)
    void lc_term(uint64_t src, uint32_t len, uint8_t coeff, uint8_t acc = 0)
    {
        Segment& s = segs_[nsegs_ - 1];
        GfOp& op = s.ops.back();
        if (len > op.n)
            len = op.n;
        if (len == 0 || coeff == 0)
            return;
        GfTerm t;
        t.src = src;
        t.len = len;
        t.coeff = coeff;
        t.acc = acc;
        t.pad = 0;
        s.terms.push_back(t);
        ++op.termCount;
    }
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
    /// (valid in this program's completion callbacks of the flush that runs it).
    uint32_t solve(const std::vector<SolveRow>& rows, const uint8_t* coef, uint32_t maxBytes);

    /// Run `fn(results)` once the next flush has completed.
    void on_complete(Completion fn);

    /// Siamese row batches (OP_ROWS, ops.h).  A batch holds a snapshot of
    /// the codec's window (elements [base, end)), lane-sum updates and rows.
    /// Any other op closes the open batch.  Protocol for the owner:
    ///   rows_window(lo, hi) -> entries to fill for elements it returns in
    ///   [*from, hi) (a batch is opened at `lo` if none covers it);
    ///   rows_update(...)    -> a lane-sum update over window elements;
    ///   rows_row(...)       -> a row reading the 24 sums and the window.
    /// Elements are the owner's window indices; the window of an open batch
    /// must not change underneath it (owners seal before shifting indices).
    WinEntry* rows_window(uint32_t lo, uint32_t hi, uint32_t* from);
    void rows_update(unsigned sumIndex, uint64_t dst, uint32_t n, uint32_t valid, unsigned s,
                     uint32_t fromElement, uint32_t toElement);
    void rows_row(const WinEntry* sums, uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix,
                  uint32_t mask0, uint32_t mask1, unsigned row, uint32_t ldpcN,
                  uint32_t ldpcFirst, const uint8_t* lit = nullptr, uint32_t litLen = 0);
    /// Close the open batch (its window may change after this).
    void rows_seal() { rows_close(); }

    /// dst[0,len) = src[0,len) (zero tail), one of a batch of independent
    /// copies (OP_COPIES): the destinations are fresh buffers no other op of
    /// the batch touches.
    void copy(uint64_t dst, uint64_t src, uint32_t len);

    bool empty() const { return nsegs_ == 0 || (nsegs_ == 1 && segs_[0].ops.empty()); }

private:
    friend class Engine;
    struct Segment
    {
        std::vector<GfOp> ops;
        std::vector<GfTerm> terms;
        std::vector<uint8_t> rowsData;   // closed OP_ROWS blocks (ops.h layout)
        uint32_t rowsWords = 0;          // stream words of those blocks (after headers)
        uint32_t maxExtent = 0;
    };
    /// The OP_ROWS batch under construction (always the segment's last op).
    struct RowsBuild
    {
        bool open = false;
        bool haveSums = false;
        WinEntry sums[kRowSums];
        uint32_t readMask = 0;          // sums read by the batch's rows
        uint32_t base = 0;              // window element of entry 0
        std::vector<WinEntry> win;
        std::vector<SumUpdate> updates;
        int updateOf[kRowSums];         // index into updates, or -1
        std::vector<RowItem> rows;
        uint32_t maxExtent = 0;
    };
    void rows_close();   // closes the open OP_ROWS or OP_COPIES batch
    void rows_open(uint32_t base, bool keepWindow);
    std::vector<CopyItem> copies_;   // the open OP_COPIES batch (segment's last op)
    // The containers of programs that went away are kept per host thread and
    // handed to new programs, so a fresh codec starts with warm capacity.
    struct Store
    {
        std::vector<Segment> segs;
        std::vector<WinEntry> win;
        std::vector<SumUpdate> updates;
        std::vector<RowItem> rows;
    };
    static std::vector<Store>& spare_stores();
    void take_store();
    void stash_store();
    struct PendingSolve
    {
        SolveDesc desc;
        std::vector<SolveRow> rows;
        std::vector<uint8_t> coef;
    };

    void touch()
    {
        if (!shard_)
            attach();
    }
    void attach();
    void new_segment();
    void reset_after_flush();

    Engine* eng_;
    int group_;
    Shard* shard_ = nullptr;     // shard this program is queued in (null: clean)
    uint32_t resultWords_ = 0;   // result words reserved since the last flush
    size_t nsegs_ = 0;           // segments in use (capacity is kept across flushes)
    std::vector<Segment> segs_;
    std::vector<PendingSolve> solves_;   // solve k follows segment k
    std::vector<Completion> callbacks_;
    RowsBuild rb_;
};

/// Algorithmic byte accounting and flush counters.
struct EngineStats
{
    uint64_t flushes = 0, launches = 0, ops = 0, terms = 0, solves = 0, ingests = 0;
    uint64_t uploadBytes = 0;
    // Source bytes of every bulk GF op the reference codec performs for the
    // same call sequence, and bytes of recovery packets / recovered
    // originals produced.
    uint64_t refOpBytes = 0, outBytes = 0;
    uint64_t solveBytes = 0;   // the part of both done by the solve kernels
    // host time of flush assembly, device waits, completion callbacks and
    // returning released buffers to the free lists (nanoseconds)
    uint64_t assembleNs = 0, waitNs = 0, completeNs = 0, reclaimNs = 0;
    uint64_t execLaunches = 0;   // executor launches (part of `launches`)

    void add(const EngineStats& o);
};

class Engine
{
public:
    /// Process-wide engine used by both ABIs.
    static Engine* global();
    ~Engine();

    bool init(int device, const char** err);
    bool ready() const { return ready_; }

    DevBuf alloc(uint32_t bytes);
    void release(DevBuf& b);               // recycled after the next flush completes
    uint64_t bytes_in_use() const;
    uint64_t arena_bytes() const { return arenaBytes_.load(std::memory_order_relaxed); }

    /// Copy `bytes` of device memory to host memory once the next flush has
    /// executed; the data is in place after sync().
    void download(void* hostDst, uint64_t devSrc, uint32_t bytes);

    /// Launch all queued work (completing the flush in flight first).
    /// Returns false once the device has failed.
    bool flush();
    /// Wait for the flush in flight and run its completions.  On a device
    /// failure nothing of that flush is delivered (no downloads, no
    /// completions), the engine is marked failed, and every instance reports
    /// Siamese_Disabled from then on (sticky, like the reference's
    /// EmergencyDisabled, siamese.h:147-150).
    bool sync();
    bool flush_and_sync()
    {
        const bool ok = flush();
        return sync() && ok;
    }
    /// A device operation failed; the engine accepts no further work.
    bool failed() const { return failed_.load(std::memory_order_relaxed); }
    bool pending() const;

    /// Copy device ranges into one host buffer right now (after completing
    /// any flush in flight).  Queued, unflushed work is not touched.
    bool gather(unsigned count, const void* const* srcs, const unsigned* bytes, void* hostOut);

    /// Serialises the drop-in siamese.h entry points and the exclusive
    /// siamese_gpu.h calls.
    std::mutex& mutex() { return mu_; }

    /// Counts toward the calling thread's statistics.
    void account(uint64_t opBytes, uint64_t outBytes = 0, bool inSolve = false);
    /// Totals over all threads.
    EngineStats stats() const;

    /// The calling thread's shard.
    Shard& shard();

private:
    friend class Program;
    void stage_host_ingest(const DevBuf& dst, const void* data, uint32_t bytes, const uint8_t* hdr,
                           uint32_t hdrLen);
    void add_ingest(const IngestDesc& d, int64_t hostStageOffset);
    uint8_t* carve_region(size_t bytes);
    bool refill(Shard& s, size_t cls, uint32_t cap);
    void spill(Shard& s);
    WorkerPool& pool();

    bool ready_ = false;
    std::atomic<bool> failed_{false};
    std::mutex mu_;

    // ---- arena: 64 MiB hipMalloc chunks are cut into 4 MiB regions under
    // arenaMu_; a shard bump-allocates buffers from its own region.  Free
    // buffers live in per-shard lists by capacity class and move between
    // shards in magazines of kMagazine through the depot (depotMu_), so a
    // buffer released on one host thread is reused on another without a
    // lock per buffer and the arena stops growing once warm.
    struct Chunk
    {
        uint8_t* base;
        size_t size, used;
    };
    std::mutex arenaMu_;
    std::vector<Chunk> chunks_;
    std::atomic<uint64_t> arenaBytes_{0};
    std::mutex depotMu_;
    std::vector<std::vector<uint8_t*>> depot_;   // [class] -> free buffers

    // ---- shards (one per host thread that touched the engine)
    mutable std::mutex shardsMu_;
    std::vector<std::unique_ptr<Shard>> shards_;

    // ---- flush-level state (exclusive)
    EngineStats flushStats_;
    struct InFlight
    {
        struct Download
        {
            void* host;
            size_t off;
            uint32_t bytes;
        };
        std::vector<Download> downloads;
        // per program: (results base, its completions in order)
        std::vector<std::pair<uint32_t, std::vector<Completion>>> callbacks;
        bool active = false;
    } flight_;
    std::unique_ptr<WorkerPool> pool_;

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

/// Per-host-thread engine state.  Only its owning thread touches it between
/// flushes, except `dirty`, which a program's destructor may edit from
/// another thread (guarded by `mu`).
struct Shard
{
    struct IngestRec
    {
        IngestDesc d;
        int64_t hostOffset;   // >= 0: src lives in this shard's host staging area
    };
    struct Download
    {
        void* host;
        uint64_t dev;
        uint32_t bytes;
    };

    std::mutex mu;
    std::vector<Program*> dirty;
    std::vector<IngestRec> ingest;
    std::vector<uint8_t> hostStage;
    std::vector<Download> downloads;
    std::vector<DevBuf> pendingFree;   // released since the last flush
    std::vector<DevBuf> flightFree;    // released before the flush in flight
    std::vector<std::vector<uint8_t*>> freeLists;   // by capacity class
    uint8_t* bump = nullptr;                         // this shard's arena region
    size_t bumpLeft = 0;
    int64_t inUse = 0;
    EngineStats stats;
};

} // namespace sgpu
