// engine.h -- device-side resources of the codec: an arena of symbol
// buffers in HBM, per-instance op programs, and the asynchronous flush
// pipeline that turns all pending programs into a handful of kernel launches.
//
// Threading: codec instances may be driven concurrently from different host
// threads (one thread per instance at a time).  Everything an instance call
// touches in the engine lives in the calling thread's Shard (buffer free
// lists, ingest queue, downloads, statistics) or in the instance's own
// Program, so per-instance calls take no global lock.
//
// Flushes are pipelined: enqueue() detaches every
// queued program body and per-thread queue in O(programs) pointer swaps and
// returns a ticket; a launcher thread lays the work out, uploads it and
// launches the kernels; a completer thread waits for the device and runs the
// completions.  enqueue() is exclusive with instance calls; wait(ticket) is
// not, so host threads keep driving other instances while a flush is
// assembled, runs on the GPU and completes.  An instance with work in a
// submission is not called again until that submission has been waited for.
#pragma once

#include "ops.h"

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <pthread.h>
#include <shared_mutex>
#include <thread>
#include <vector>

namespace sgpu {

/// The drop-in API's instance lock: a reader-writer lock that prefers the
/// writer.  Instance calls hold it shared for microseconds; a flush holds it
/// exclusively only to detach the queued work.  std::shared_mutex (glibc's
/// default rwlock) prefers readers, so with many application threads calling
/// in, a flush's exclusive request waited behind an unbroken stream of
/// instance calls.  The readers count themselves in per-thread slots (a
/// cache line each): a shared acquisition touches no line another thread
/// writes, where one rwlock word bounced between every calling core (the
/// drop-in's 0.1 us adds took 0.55 us each from 16 threads,
/// profiles/r5k_dropin_calls_16threads.txt).  A writer raises its flag and
/// waits for every slot to drain; readers that see the flag step back and
/// wait for it to drop.  Never taken shared twice by one thread (a waiting
/// writer would block the second acquisition): builds with SGPU_DEBUG_LOCKS
/// abort on a nested shared acquisition (tests/instance_lock_test.cpp is
/// built so).  Unlike glibc's rwlock it is not re-entrant and prefers the
/// writer, so no instance call may wait on a flush while it holds the lock
/// shared (the flush's detach takes it exclusively): the decoder and encoder
/// mirror paths return kNeedsFlush instead and flush outside it.
class InstanceLock
{
public:
    InstanceLock() = default;
    InstanceLock(const InstanceLock&) = delete;
    InstanceLock& operator=(const InstanceLock&) = delete;
    void lock()
    {
        wmu_.lock();   // (one writer at a time)
        writer_.store(1, std::memory_order_seq_cst);
        for (Slot& s : slots_)
            for (unsigned spin = 0; s.n.load(std::memory_order_seq_cst) != 0; ++spin)
                pause(spin);
    }
    bool try_lock()
    {
        if (!wmu_.try_lock())
            return false;
        writer_.store(1, std::memory_order_seq_cst);
        for (Slot& s : slots_)
            if (s.n.load(std::memory_order_seq_cst) != 0) {
                unlock();
                return false;
            }
        return true;
    }
    void unlock()
    {
        writer_.store(0, std::memory_order_seq_cst);
        wmu_.unlock();
        if (waiters_.load(std::memory_order_seq_cst) != 0) {
            std::lock_guard<std::mutex> g(cvMu_);
            cv_.notify_all();
        }
    }
    void lock_shared()
    {
        debug_enter();
        std::atomic<int>& n = slot();
        for (;;) {
            n.fetch_add(1, std::memory_order_seq_cst);
            if (writer_.load(std::memory_order_seq_cst) == 0)
                return;
            n.fetch_sub(1, std::memory_order_seq_cst);
            wait_writer();
        }
    }
    bool try_lock_shared()
    {
        debug_enter();
        std::atomic<int>& n = slot();
        n.fetch_add(1, std::memory_order_seq_cst);
        if (writer_.load(std::memory_order_seq_cst) == 0)
            return true;
        n.fetch_sub(1, std::memory_order_seq_cst);
        debug_leave();
        return false;
    }
    void unlock_shared()
    {
        slot().fetch_sub(1, std::memory_order_release);
        debug_leave();
    }

private:
#ifdef SGPU_DEBUG_LOCKS
    static int& depth()
    {
        thread_local int d = 0;
        return d;
    }
    static void debug_enter()
    {
        if (depth()++ != 0) {
            std::fprintf(stderr, "InstanceLock: nested shared acquisition\n");
            std::abort();
        }
    }
    static void debug_leave() { --depth(); }
#else
    static void debug_enter() {}
    static void debug_leave() {}
#endif
    static constexpr unsigned kSlots = 64;
    struct alignas(64) Slot
    {
        std::atomic<int> n{0};
    };
    std::atomic<int>& slot()
    {
        static std::atomic<unsigned> next{0};
        thread_local const unsigned mine = next.fetch_add(1, std::memory_order_relaxed) % kSlots;
        return slots_[mine].n;
    }
    static void pause(unsigned spin)
    {
        if (spin < 256)
            __builtin_ia32_pause();
        else
            std::this_thread::yield();
    }
    void wait_writer()
    {
        // a detach takes microseconds: spin first, then sleep until unlock()
        for (unsigned spin = 0; spin < 512; ++spin) {
            if (writer_.load(std::memory_order_seq_cst) == 0)
                return;
            __builtin_ia32_pause();
        }
        std::unique_lock<std::mutex> lk(cvMu_);
        waiters_.fetch_add(1, std::memory_order_seq_cst);
        cv_.wait(lk, [&] { return writer_.load(std::memory_order_seq_cst) == 0; });
        waiters_.fetch_sub(1, std::memory_order_relaxed);
    }

    Slot slots_[kSlots];
    alignas(64) std::atomic<int> writer_{0};
    std::atomic<int> waiters_{0};
    std::mutex wmu_;
    std::mutex cvMu_;
    std::condition_variable cv_;
};

class WorkerPool;

/// A symbol-sized buffer in device memory.  Capacity is a multiple of 64 B.
struct DevBuf
{
    uint8_t* ptr = nullptr;
    uint32_t cap = 0;
    explicit operator bool() const { return ptr != nullptr; }
    uint64_t addr() const { return (uint64_t)(uintptr_t)ptr; }
};

/// Buffer capacity for `bytes` (64 B classes up to 4 KiB, 1 KiB classes up
/// to 128 KiB, 64 KiB classes above).
uint32_t round_cap(uint32_t bytes);

/// The originals of one subwindow (64 consecutive window elements) live in
/// one slab: 64 slots of one capacity, taken whole from the arena when the
/// subwindow's first original arrives and released whole when the
/// subwindow leaves the window (the reference recycles whole subwindows,
/// SiameseEncoder.cpp:284-315).  Consecutive originals then fill
/// consecutive slots, so a run of adds is one ingest descriptor and one
/// allocation.  A slot is written at most once per slab: a later symbol for
/// it (or one too large for the stride) gets a buffer of its own, since
/// ops of the same flush may still read the slot's first contents.
struct Slab
{
    DevBuf buf;
    uint32_t stride = 0;
    uint64_t used = 0;   // slots written since the slab was taken
};

class Engine;
struct Shard;
struct Batch;

/// Completion callback of a flush; `results` is the solve-result word array
/// as seen by the program that registered it (indices returned by solve()).
using Completion = std::function<void(const uint32_t* results)>;

/// Everything a program has queued since it was last detached.  Bodies move
/// whole into a flush (an O(1) swap) and come back to a shared pool once the
/// flush has been laid out and completed, keeping their capacity.
struct ProgramBody
{
    struct Segment
    {
        std::vector<GfOp> ops;
        std::vector<GfTerm> terms;
        std::vector<uint8_t> rowsData;   // closed OP_ROWS / OP_COPIES blocks (ops.h layout)
        uint32_t rowsWords = 0;          // stream words of those blocks (after headers)
        uint32_t maxExtent = 0;
        /// Wide rows of the closed OP_ROWS blocks, whose LDPC picks k_ldpc
        /// computes (ops.h LdpcItem): filled in at flush assembly.
        struct Wide
        {
            uint32_t op;       // index into ops (the OP_ROWS header)
            uint32_t entry;    // window index of its L0 entry (L1 follows)
            uint32_t n, row, N, off;
        };
        std::vector<Wide> wide;
        uint32_t wideItems = 0;          // k_ldpc items of those rows
        uint64_t wideBytes = 0;          // scratch bytes of those rows
        /// Ops gated on a chained matrix job's outcome (ops.h GeDesc
        /// kGeChained): ops [opBegin, opEnd) run only if the body's result
        /// word `word` is non-zero (the header's termBegin on the device,
        /// made absolute at assembly)
        struct Gate
        {
            uint32_t opBegin, opEnd, word;
        };
        std::vector<Gate> gates;
        void clear()
        {
            ops.clear();
            terms.clear();
            rowsData.clear();
            rowsWords = 0;
            maxExtent = 0;
            wide.clear();
            wideItems = 0;
            wideBytes = 0;
            gates.clear();
        }
    };
    /// The OP_ROWS batch under construction (always the segment's last op).
    struct RowsBuild
    {
        bool open = false;
        bool haveSums = false;
        uint64_t sumsVersion = 0;       // the caller's table `sums` was copied from (0: none)
        WinEntry sums[kRowSums];
        uint32_t readMask = 0;          // sums read by the batch's rows
        uint32_t cutMax = 0;            // largest row cutoff so far (absolute element)
        bool versioned = false;         // an update joined after a row read its sum
        uint32_t base = 0;              // window element of entry 0
        std::vector<WinEntry> win;
        std::vector<SumUpdate> updates;
        int updateOf[kRowSums];         // index into updates, or -1
        std::vector<RowItem> rows;
        uint32_t maxExtent = 0;
    };
    struct PendingSolve
    {
        SolveDesc desc;
        std::vector<SolveRow> rows;
        std::vector<uint8_t> coef;
        // where assembly placed its rows and coefficients (a chained matrix
        // job of the same body writes them there, GeDesc.solveRow/solveCoef)
        mutable uint32_t asmRow = 0, asmCoef = 0;
    };
    /// A device matrix generation + elimination (ops.h GeDesc): its input
    /// as k_ge reads it and its first result word.
    struct PendingGe
    {
        uint16_t rows = 0, cols = 0;
        uint32_t pickLen = 0;
        uint32_t result = 0;
        bool chained = false;   // kGeChained: feeds solves[solve] of the same body
        uint32_t solve = 0;
        std::vector<uint8_t> in;
    };

    int group = 0;
    uint32_t resultWords = 0;   // result words reserved in this body
    size_t nsegs = 0;           // segments in use (capacity is kept)
    std::vector<Segment> segs;
    std::vector<PendingSolve> solves;   // solve k follows segment k (nsolves in use)
    size_t nsolves = 0;
    std::vector<PendingGe> ges;         // independent of the segments (nges in use)
    size_t nges = 0;
    std::vector<Completion> callbacks;
    // objects the callbacks use, kept alive until they have run (so a
    // callback captures a raw pointer and fits std::function's inline
    // storage: no heap block per callback)
    std::vector<std::shared_ptr<void>> keep;
    RowsBuild rb;
    bool gateOpen = false;        // ops from (segment gateSeg, op gateOp) on are gated on gateWord
    size_t gateSeg = 0;
    uint32_t gateOp = 0, gateWord = 0;
    std::vector<CopyItem> copies;       // the open OP_COPIES batch (segment's last op)
    /// The open OP_LINCOMBS batch (ops.h): independent combinations waiting
    /// to be sealed as one op after the segment's last op.
    struct LcBuild
    {
        std::vector<LcItem> items;
        std::vector<GfTerm> terms;   // termStart: index into this, made block-relative on seal
        /// Byte spans written / read by every item but the last, each set
        /// disjoint and sorted (the independence tests are binary searches;
        /// the last item stays out until the next one joins, because a footer
        /// literal may still grow its write span).
        struct Span
        {
            uint64_t lo, hi;
        };
        std::vector<Span> writes, reads;
        void clear()
        {
            items.clear();
            terms.clear();
            writes.clear();
            reads.clear();
        }
    } lcb;
    std::vector<GfTerm> lcScratch;
    void lc_seal();                     // seals the open OP_LINCOMBS batch
    /// Move the segment's last op (an OP_LINCOMB) into the open batch, or
    /// seal the batch first when they are not independent.
    void lc_absorb();
    /// May a literal at [at, at + len) join the batch's last item?
    bool lc_literal_fits(uint64_t at, uint32_t len) const;

    bool empty() const
    {
        return nges == 0 &&
               (nsegs == 0 ||
                (nsegs == 1 && segs[0].ops.empty() && copies.empty() && lcb.items.empty() && !rb.open));
    }
    void new_segment();
    void rows_open(uint32_t base, bool keepWindow);
    void rows_close();   // closes the open OP_ROWS or OP_COPIES batch
    void clear();        // back to the freshly constructed state (capacity kept)

    static ProgramBody* get();
    static void put(ProgramBody* b);
};

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
    // (lc_term must follow lc_begin directly: it appends to the last op)
    void lc_term(uint64_t src, uint32_t len, uint8_t coeff, uint8_t acc = 0)
    {
        ProgramBody::Segment& s = b_->segs[b_->nsegs - 1];
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
    /// `count` symbols of one shape: symbol k from src + k * srcStride into
    /// the fresh slot dst + k * dstStride (IngestDesc runs).
    void ingest_run(uint64_t dst, uint32_t dstStride, uint64_t src, uint32_t srcStride, uint32_t count,
                    uint32_t bytes, const uint8_t* hdr, uint32_t hdrLen);

    /// Queue a triangular solve; returns the result-word index it will fill
    /// (valid in this program's completion callbacks of the flush that runs it).
    uint32_t solve(const std::vector<SolveRow>& rows, const uint8_t* coef, uint32_t maxBytes);
    /// solve() in two halves, without the copies: solve_reserve hands out the
    /// queued solve's own row descriptors (m) and coefficients (m x m) to
    /// fill; solve_commit queues it (same result word as solve()).  No other
    /// solve may be queued in between.
    void solve_reserve(unsigned m, SolveRow** rows, uint8_t** coef);
    /// gateWord (optional, 1 + a result word): the solve runs only if that
    /// word is non-zero, on the coefficients and row order the program's
    /// last chained matrix job writes (ge_job chained).
    uint32_t solve_commit(uint32_t maxBytes, uint32_t gateWord = 0);

    /// Queue a device matrix generation + elimination (ops.h GeDesc) of
    /// rows x cols with a pick table of pickLen bytes: returns the job's
    /// input buffer (ge_input_bytes, for the caller to fill before the next
    /// flush) and *resultWord, its first result word (valid in this
    /// program's completion callbacks).  chained (rows == cols): the next
    /// solve this program queues is the decode's, and the job writes its
    /// coefficients and row order (solve_commit with the job's gate).
    uint8_t* ge_job(unsigned rows, unsigned cols, unsigned pickLen, uint32_t* resultWord, bool chained = false);
    /// Gate every op queued from now until gate_end() on result word `word`:
    /// they run only if it is non-zero (a chained matrix job's outcome, ops.h
    /// GeDesc word 3).  No solve and no literal may be queued in between.
    void gate_begin(uint32_t word);
    void gate_end();

    /// Run `fn(results)` once the flush holding this program's work completes.
    /// Callbacks of one flush run in registration order on one thread, but
    /// callbacks of different flushes may run concurrently and out of ticket
    /// order (an inline flush's caller completes its own submission while the
    /// completer thread completes the next one; only the tickets' publication
    /// is ordered).  A callback may therefore touch only state keyed by its
    /// own submission -- the decoder's Resolver slots under Resolver::mu
    /// (complete_solve) -- never state a later flush's callback also writes.
    void on_complete(Completion fn);
    /// on_complete, `keep` held until the callback has run.
    void on_complete(std::shared_ptr<void> keep, Completion fn);
    /// Forget the completions of work not yet submitted (owner going away).
    void drop_callbacks()
    {
        if (b_) {
            b_->callbacks.clear();
            b_->keep.clear();
        }
    }

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
    /// `cutoff`: the row reads each sum as folded over window elements below
    /// it (every sum the row reads was brought up to it; RowItem.cutoff).
    /// `sumsVersion` (optional, from next_table_version()): the caller's
    /// table has not changed since a row passed it with this version, so
    /// the batch's copy is not compared or copied again.
    void rows_row(const WinEntry* sums, uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix,
                  uint32_t mask0, uint32_t mask1, unsigned row, uint32_t ldpcN,
                  uint32_t ldpcFirst, uint32_t cutoff, const uint8_t* lit = nullptr, uint32_t litLen = 0,
                  uint64_t sumsVersion = 0);
    /// A fresh version tag for a caller's sums table (rows_row), unique in the process.
    static uint64_t next_table_version();
    /// Close the open batch (its window may change after this).
    void rows_seal()
    {
        if (b_)
            b_->rows_close();
    }

    /// dst[0,len) = src[0,len) (zero tail), one of a batch of independent
    /// copies (OP_COPIES): the destinations are fresh buffers no other op of
    /// the batch touches.
    void copy(uint64_t dst, uint64_t src, uint32_t len);

    bool empty() const { return !b_ || b_->empty(); }

private:
    friend class Engine;
    void touch()
    {
        if (!shard_)
            attach();
    }
    void attach();
    void rows_open(uint32_t base, bool keepWindow) { b_->rows_open(base, keepWindow); }

    Engine* eng_;
    int group_;
    Shard* shard_ = nullptr;     // shard this program is queued in (null: clean)
    ProgramBody* b_ = nullptr;   // the queued work (null until the first op)
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
    uint64_t ldpcBytes = 0;    // the part of refOpBytes done by k_ldpc (wide rows' picks)
    // host time of flush assembly (launcher thread), device waits and
    // completion callbacks (completer thread), and returning released
    // buffers to the arena (nanoseconds)
    uint64_t assembleNs = 0, waitNs = 0, completeNs = 0, reclaimNs = 0;
    uint64_t execLaunches = 0;   // executor launches (part of `launches`)
    // Compulsory bytes of the executor launches, counted only while
    // set_measure_unique(true) (bench.py's roofline): every distinct source
    // symbol read once, every destination written once, plus the op stream.
    uint64_t execUniqueBytes = 0;
    // device recovery-matrix jobs (sgpu_decode_device): all, chained into
    // their decode's submission, chained ones that found a singular matrix
    uint64_t geJobs = 0, geChained = 0, geRetried = 0;

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
    /// Slot `bit` of the slab for a symbol of `need` bytes (the slab is
    /// taken on first use), or a null buffer when it cannot hold it (taken
    /// slot, too large, slabs off); *failed on an arena failure.
    DevBuf slab_slot(Slab& sl, unsigned bit, uint32_t need, bool* failed);
    void slab_release(Slab& sl)
    {
        release(sl.buf);
        sl.stride = 0;
        sl.used = 0;
    }
    uint64_t bytes_in_use() const;
    uint64_t arena_bytes() const { return arenaBytes_.load(std::memory_order_relaxed); }
    /// Keep at least `bytes` of untouched arena chunks in reserve, so later
    /// growth takes them instead of calling hipMalloc (an application calls
    /// this before a latency-sensitive phase).  False if hipMalloc fails.
    bool reserve(size_t bytes);

    /// Copy `bytes` of device memory to host memory once the next flush has
    /// executed; the data is in place after that flush has been waited for.
    void download(void* hostDst, uint64_t devSrc, uint32_t bytes);

    /// Detach all queued work and hand it to the launcher.  Exclusive with
    /// instance calls.  Returns the submission's ticket (> 0), or 0 once the
    /// device has failed.
    uint64_t enqueue();
    /// Wait until submission `ticket` (and every earlier one) has completed.
    /// On a device failure nothing of the failed submission is delivered (no
    /// downloads, no completions), the engine is marked failed, and every
    /// instance reports Siamese_Disabled from then on (sticky, like the
    /// reference's EmergencyDisabled, siamese.h:147-150).
    bool wait(uint64_t ticket);
    /// Non-blocking: has submission `ticket` completed?
    bool done(uint64_t ticket)
    {
        std::lock_guard<std::mutex> g(qMu_);
        return doneTicket_ >= ticket;
    }
    /// Ticket of the latest submission.
    uint64_t last_ticket() const { return nextTicket_.load(std::memory_order_acquire); }
    /// Submit, then complete the previous submission (one flush in flight).
    bool flush();
    /// Complete every submission.
    bool sync() { return wait(nextTicket_.load(std::memory_order_acquire)); }
    /// Submit everything queued and wait for it.  With nothing in flight
    /// the caller's thread runs the submission itself (assembly, launches,
    /// fence poll, completion): no hand-off to the launcher and completer
    /// threads, the drop-in siamese.h path's per-call latency.  detach: a
    /// lock that instance calls hold shared (the drop-in API's), held
    /// exclusively while the queued work is detached; concurrent callers
    /// commit as a group (the first one's submission carries everything
    /// queued before it, the others find their work taken and only wait).
    bool flush_and_sync(InstanceLock* detach = nullptr);
    /// A device operation failed; the engine accepts no further work.
    bool failed() const { return failed_.load(std::memory_order_relaxed); }
    bool pending() const;

    /// Copy device ranges into one host buffer right now (after completing
    /// every submission).  Queued, unsubmitted work is not touched.
    bool gather(unsigned count, const void* const* srcs, const unsigned* bytes, void* hostOut);
    /// Gather ranges written by COMPLETED submissions into pinned host memory
    /// on the gather stream, without waiting for submissions in flight.
    /// Range i lands at the 16-byte aligned running offset (see
    /// sgpu_gather_completed).
    bool gather_completed(unsigned count, const void* const* srcs, const unsigned* bytes, void* pinnedOut);
    /// The same without waiting for the copy: returns a gather ticket (> 0,
    /// or -1 on failure).  The sources are read before any later submission's
    /// device work runs (it waits for them on the device), so the caller may
    /// go on driving the instances that own them; pinnedOut is filled once
    /// gather_wait(ticket) returns true.
    int64_t gather_async(unsigned count, const void* const* srcs, const unsigned* bytes, void* pinnedOut);
    /// The same with a header of hdrLens[i] <= 8 bytes (hdrs + 8 i) written
    /// before range i: range i lands at the running offset of
    /// align16(hdrLens[k] + bytes[k]) over k < i, zero-padded (framed egress).
    int64_t gather_async_framed(unsigned count, const void* const* srcs, const unsigned* bytes,
                                const uint8_t* hdrs, const unsigned* hdrLens, void* pinnedOut);
    /// Wait until gather `ticket` and every earlier one have landed.
    bool gather_wait(int64_t ticket);
    /// Host -> device copy on the staging stream, issued now; every later
    /// submission's device work waits for it (the host does not).  The caller
    /// guarantees that no unfinished submission touches dst.
    bool stage_in(void* dst, const void* src, size_t bytes);

    /// Serialises the exclusive siamese_gpu.h calls.
    std::mutex& mutex() { return mu_; }
    /// Shared by the drop-in siamese.h instance calls (each instance used by
    /// one thread at a time; concurrent calls on different instances are this
    /// library's extension of siamese.h:59), exclusive only while a flush
    /// detaches the queued work (flush_and_sync(&instance_lock())).
    InstanceLock& instance_lock() { return instMu_; }

    /// Count EngineStats::execUniqueBytes at flush assembly (a measurement
    /// aid: off by default, it sorts every segment's operands).
    static void set_measure_unique(bool on);
    static bool measure_unique();

    /// Counts toward the calling thread's statistics.
    void account(uint64_t opBytes, uint64_t outBytes = 0, bool inSolve = false);
    /// Totals over all threads.
    EngineStats stats() const;

    /// The calling thread's shard.
    Shard& shard();

    /// The engine's host worker pool (also offered to applications,
    /// sgpu_parallel_for).
    WorkerPool& pool();

private:
    friend class Program;
    void stage_host_ingest(const DevBuf& dst, const void* data, uint32_t bytes, const uint8_t* hdr,
                           uint32_t hdrLen);
    void add_ingest(const IngestDesc& d, int64_t hostStageOffset);
    uint8_t* carve_region(size_t bytes);
    bool refill(Shard& s, size_t cls, uint32_t cap);

    // ---- flush pipeline
    void launcher_loop();
    void completer_loop();
    void assemble_batch(Batch& b, WorkerPool& wp);
    Batch* take_batch();   // queued programs and queues as a batch with its ticket (nullptr: none)
    void claim_set(Batch& b);
    bool flush_requested(std::unique_lock<std::mutex>& sub, InstanceLock& detach);
    bool run_inline(Batch* b, std::unique_lock<std::mutex>& sub);
    Batch* take_requested();   // launcher thread: detach for filed flush requests
    WorkerPool& asm_pool();   // launcher thread only
    void launch_batch(Batch& b);
    bool complete_batch(Batch& b);   // false: the submission failed
    void reclaim_batch(Batch& b);    // released buffers to the depot (before the ticket is published)
    void start_threads();
    void stop_threads();

    bool ready_ = false;
    std::atomic<bool> failed_{false};
    std::mutex mu_;
    InstanceLock instMu_;
    // one submission detached and assembled at a time (take_batch hands out
    // tickets, and toLaunch_ keeps ticket order); held by enqueue() and
    // flush_and_sync() until the batch is queued or launched
    std::mutex submitMu_;

    // ---- arena: 64 MiB hipMalloc chunks are cut into 4 MiB regions under
    // arenaMu_; a shard bump-allocates buffers from its own region.  Free
    // buffers live in per-shard lists by capacity class; a completed flush
    // returns its released buffers to the depot (depotMu_) in magazines,
    // which shards take whole when their list runs dry, so the arena stops
    // growing once warm.
    struct Chunk
    {
        uint8_t* base;
        size_t size, used;
    };
    std::mutex arenaMu_;
    std::vector<Chunk> chunks_;
    std::vector<Chunk> spare_;   // reserved ahead, not yet carved
    std::atomic<uint64_t> arenaBytes_{0};
    std::mutex depotMu_;
    struct Magazine
    {
        uint64_t ticket = 0;          // the submission that released these buffers
        std::vector<uint8_t*> bufs;
    };
    std::vector<std::vector<Magazine>> depot_;   // [class] -> magazines

    // ---- shards (one per host thread that touched the engine)
    mutable std::mutex shardsMu_;
    std::vector<std::unique_ptr<Shard>> shards_;

    // ---- flush pipeline state
    std::mutex statsMu_;
    EngineStats flushStats_;
    std::atomic<uint64_t> nextTicket_{0};           // last ticket handed out (take_batch, under submitMu_)
    std::mutex qMu_;
    std::condition_variable launchCv_, completeCv_, doneCv_, setCv_;
    std::deque<Batch*> toLaunch_, toComplete_;
    std::vector<void*> pendingMarks_;               // staged copies the next submission waits for (qMu_)
    std::mutex gatherMu_;
    uint64_t doneTicket_ = 0;                       // every ticket <= this has completed
    // lock-free mirrors for the short spins before blocking (single-stream
    // latency: a flush is a few tens of microseconds of device work, less
    // than a futex wake-up of the launcher plus one of the waiting caller)
    std::atomic<uint64_t> doneSeen_{0};             // doneTicket_
    std::atomic<uint64_t> queuedSeen_{0};           // batches pushed to toLaunch_
    bool stop_ = false;
    bool launching_ = false;                        // the launcher holds a batch (qMu_)
    // drop-in flush requests (qMu_): filed, and covered by the launcher's
    // latest detach, whose last ticket is reqTicket_
    uint64_t flushReq_ = 0;
    uint64_t takenReq_ = 0;
    uint64_t reqTicket_ = 0;
    bool completing_ = false;                       // the completer holds a batch (qMu_)
    bool inlineBusy_ = false;                       // a caller runs a submission itself (qMu_)
    std::thread launcher_, completer_;
    std::unique_ptr<WorkerPool> pool_;
    std::unique_ptr<WorkerPool> asmPool_;

    // transfer buffer sets: one per submission in flight (ticket % kSets)
    static constexpr unsigned kSets = 4;
    struct XferSet
    {
        uint8_t* upHost = nullptr;
        uint8_t* upDev = nullptr;
        uint8_t* upHostDev = nullptr;   // upHost as the device addresses it (zero-copy), or null
        size_t upCap = 0;
        uint8_t* downHost = nullptr;
        uint8_t* downDev = nullptr;   // device-side gather area for downloads + results
        uint8_t* downHostDev = nullptr;   // downHost as the device addresses it, or null
        size_t downCap = 0;
        uint64_t busyTicket = 0;      // submission using it (0: free)
        uint8_t* wideDev = nullptr;   // k_ldpc scratch ring (see ensure_wide)
        size_t wideCap = 0;
        size_t wideUsed = 0;          // bytes of the ring dirtied since it was zeroed
        // the product solves' inverses and results (written before they are
        // read within a submission: reused from its start, never zeroed)
        uint8_t* solveDev = nullptr;
        size_t solveCap = 0;
        // the device byte counters at the head of downDev only grow (no
        // memset per submission): each completion takes the difference
        uint64_t acctPrev[4] = {0, 0, 0, 0};
        bool acctZero = false;        // fresh downDev: zero the counters first
    } sets_[kSets];
    void ensure_up(XferSet& x, size_t bytes);
    void ensure_wide(XferSet& x, size_t bytes);
    void ensure_solve(XferSet& x, size_t bytes);
    void ensure_down(XferSet& x, size_t bytes);

    // gather buffers (separate from the flush buffers)
    uint8_t* gUpHost_ = nullptr;
    uint8_t* gUpDev_ = nullptr;
    size_t gUpCap_ = 0;
    uint8_t* gHost_ = nullptr;
    uint8_t* gDev_ = nullptr;
    size_t gCap_ = 0;
    // gather_async slots, one per gather in flight (gatherMu_): descriptor
    // upload and packing area, reused once the slot's previous gather landed
    static constexpr unsigned kGatherSlots = 4;
    struct GatherSlot
    {
        uint8_t* upHost = nullptr;
        uint8_t* upDev = nullptr;
        size_t upCap = 0;
        uint8_t* stage = nullptr;
        size_t stageCap = 0;
        void* landed = nullptr;   // mark passed once the host bytes are in place
        int64_t ticket = 0;
    } gslots_[kGatherSlots];
    int64_t gNext_ = 0;
    bool gather_land(GatherSlot& g);
};

/// Per-host-thread engine state.  Only its owning thread touches it between
/// submissions, except `dirty`, which a program's destructor may edit from
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
    /// What a submission takes from the shard (swapped out whole).
    struct Queues
    {
        std::vector<IngestRec> ingest;
        std::vector<uint8_t> hostStage;
        std::vector<Download> downloads;
        std::vector<std::vector<uint8_t*>> released;   // by capacity class
        uint32_t maxIngest = 0;                         // largest hdrLen + bytes among `ingest`
        size_t pairCursor = 0;                          // ingest run a decoder's symbols paired with last
        bool empty() const;
        void clear();
    };

    std::mutex mu;
    std::vector<Program*> dirty;
    Queues q;
    std::vector<Queues> spare;                      // recycled by completed submissions (mu)
    std::vector<std::vector<uint8_t*>> freeLists;   // by capacity class
    uint8_t* bump = nullptr;                        // this shard's arena region
    size_t bumpLeft = 0;
    int64_t inUse = 0;
    EngineStats stats;
};

} // namespace sgpu
