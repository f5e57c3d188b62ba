// decoder.h -- host control plane of the decoder.
//
// The bookkeeping (receive window, recovery list ordering, checked region,
// matrix generation and Gaussian elimination on coefficients) mirrors the
// reference decoder so decode timing and results are identical
// (reference SiameseDecoder.h:108-632, SiameseDecoder.cpp:255-2700).
// Symbol work -- eliminating received originals, lane sums, the triangular
// solve -- is emitted as device ops; coefficients never leave the host.
//
// Recovered lengths are only known once the device has solved the length
// prefix.  Until then a recovered slot carries an UPPER BOUND (its recovery
// row's length) with the device guaranteeing zeros beyond the true length,
// which makes every later op numerically identical; the exact value is
// patched in when the flush completes (see resolve()).
#pragma once

#include "codedef.h"
#include "encoder.h"
#include "engine.h"
#include "gf.h"
#include "objpool.h"
#include "../../include/siamese.h"

#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

namespace sgpu {

/// decode_device: a matrix job was queued; call again after the flush
/// (siamese_gpu.h SGPU_DECODE_PENDING)
constexpr SiameseResult kDecodePending = static_cast<SiameseResult>(6);
/// DecoderCore::get in drop-in (mirror) mode: the packet's exact length is
/// still on the device; flush outside the instance lock and call again
constexpr SiameseResult kNeedsFlush = static_cast<SiameseResult>(7);

struct DecSlot
{
    DevBuf buf;
    bool inSlab = false;        // buf is a slot of the subwindow's slab (not owned)
    unsigned bytes = 0;         // prefix + payload (upper bound while pending)
    unsigned column = 0;        // packet number, or matrix column while lost
    unsigned header = 0;
    bool pending = false;       // recovered, exact length not yet known
    uint32_t pendSlot = 0;      // while pending: the solve that recovers it (Resolver::pend index)
    uint32_t pendCi = 0;        //   and its column within that solve
    // host mirror (drop-in mode only): out of line, so the batch path's
    // window scans touch a 48-byte slot
    std::unique_ptr<std::vector<uint8_t>> hostp;
    std::vector<uint8_t>& host()
    {
        if (!hostp)
            hostp.reset(new std::vector<uint8_t>);
        return *hostp;
    }
};

struct DecSubwindow
{
    DecSlot slot[kSubwindow];
    uint64_t got = 0;           // CustomBitSet<64> (PacketAllocator.h:189-437)
    unsigned gotCount = 0;
    Slab slab;                  // the received originals' shared buffer (engine.h)
    bool clean = false;         // every slot already in its fresh state (the owner's teardown)
    void reset()
    {
        got = 0;
        gotCount = 0;
        for (DecSlot& s : slot) {
            s.column = 0;
            s.bytes = 0;
            s.pending = false;
        }
    }
};

/// unique_ptr deleter: subwindows go back to the thread's pool, emptied
/// (their buffers were released by the owner).
struct DecSubwindowRecycle
{
    void operator()(DecSubwindow* w) const;
};
using DecSubwindowPtr = std::unique_ptr<DecSubwindow, DecSubwindowRecycle>;

struct RecPacket
{
    RecPacket* next = nullptr;
    RecPacket* prev = nullptr;
    RowMeta meta;
    unsigned elementStart = 0;
    unsigned elementEnd = 0;
    unsigned lostCount = 0;
    DevBuf buf;
    unsigned bytes = 0;
};

/// Handle to a recovery packet that already lives in device memory (batch API).
struct DeviceRecovery
{
    uint64_t data = 0;          // device address of the packet (payload+footer)
    unsigned bytes = 0;
    const uint8_t* footer = nullptr;  // host copy of the footer bytes
    unsigned footerBytes = 0;
    const uint8_t* head = nullptr;    // host copy of the first bytes (single rows)
    Program* producer = nullptr;      // program that must perform the copy; null:
                                      // a staged packet (a host -> device copy the
                                      // submission waits for, any alignment)
};

class DecoderCore
{
public:
    DecoderCore(Engine* eng, bool hostMirror);
    ~DecoderCore();

    Program& program() { return prog_; }

    SiameseResult add_original(const SiameseOriginalPacket& packet, uint64_t deviceSrc = 0);
    /// `count` add_original calls in one (sgpu_decoder_add_original_range):
    /// packet firstNum + k from src + k * srcStride, lens[k] bytes (fixedBytes
    /// when lens is null).  results[k] (optional) gets each call's result;
    /// like the calls, a DuplicateData goes on and any other failure stops
    /// (its result returned, *added = calls made including it).  Consecutive
    /// slab slots become one ingest run.
    SiameseResult add_original_range(unsigned firstNum, uint64_t src, uint32_t srcStride, const unsigned* lens,
                                     unsigned fixedBytes, unsigned count, SiameseResult* results,
                                     unsigned* added);
    /// sgpu_decoder_get_range: get() for packets firstNum, firstNum + 1, ...
    /// into out[0..count) until one is not Success; *got = packets returned.
    /// Returns the result of the get that stopped (Success if none did).
    SiameseResult get_range(unsigned firstNum, unsigned count, SiameseOriginalPacket* out, unsigned* got);
    /// Host-memory recovery packet (drop-in API).
    SiameseResult add_recovery(const SiameseRecoveryPacket& packet);
    /// Device-resident recovery packet (batch API).
    SiameseResult add_recovery_device(const DeviceRecovery& rec);
    SiameseResult is_ready();
    /// Queues the solve; packets' lengths become exact after resolve().
    SiameseResult decode(SiameseOriginalPacket** packetsOut, unsigned* countOut);
    /// decode() with a fresh recovery matrix generated and eliminated on the
    /// device (sgpu_decode_device): returns kDecodePending after queueing the
    /// matrix job; the next call after the flush that ran it finishes the
    /// decode as decode() would have (an elimination that stopped short is
    /// repeated on the host, which keeps the resumable state).  A square
    /// matrix of Siamese rows of one length (a block decode) is chained: the
    /// elimination of received data and the solve go into the same
    /// submission, gated on the device elimination's outcome, so the call
    /// after the flush returns the recovered packets with their lengths.
    SiameseResult decode_device(SiameseOriginalPacket** packetsOut, unsigned* countOut);
    /// A device matrix job is queued and not yet finished by decode_device.
    bool ge_pending() const { return geState_ != 0; }
    SiameseResult get(SiameseOriginalPacket& packet);
    /// Deferred forms (siamese_gpu.h sgpu_decode_deferred /
    /// sgpu_decoder_get_deferred): never wait for the device.  Outputs go to
    /// caller-owned entries; an entry whose length is still being solved gets
    /// Data/DataBytes written when the submission carrying the solve
    /// completes (before that submission reads as done).
    SiameseResult decode_deferred(SiameseOriginalPacket* out, unsigned capacity, unsigned* countOut);
    SiameseResult get_deferred(SiameseOriginalPacket& packet);
    /// Apply completed solves to the decoder's own state (recovered slots'
    /// exact lengths, a corrupt prefix's Disabled): every call does this first.
    void settle()
    {
        if (res_->doneCount.load(std::memory_order_acquire) != appliedCount_)
            apply_resolved();
    }
    SiameseResult stats(uint64_t* out, unsigned count);
    /// ARQ: siamese_decoder_ack (arq.cpp)
    SiameseResult acknowledgement(uint8_t* buffer, unsigned byteLimit, unsigned& usedBytes);

    /// Disabled: this instance failed (sticky), or the device did (Engine::failed).
    bool disabled()
    {
        settle();
        return dead();
    }
    bool dead() const { return disabled_ || eng_->failed(); }
    /// Packet present in the window (received or recovered, length may be pending)
    bool has(unsigned packetNum)
    {
        settle();
        const unsigned e = column_to_element(packetNum);
        return !dead() && e < count_ && slot(e).bytes > 0;
    }
    /// Present, but its exact length still being solved on the device (a
    /// get() would flush and wait).
    bool pending(unsigned packetNum)
    {
        settle();
        const unsigned e = column_to_element(packetNum);
        return !dead() && e < count_ && slot(e).bytes > 0 && slot(e).pending;
    }
    /// True while a queued solve has not been resolved by a completed flush.
    bool has_pending() const { return pendingSolves_ > 0; }
    /// Drop-in mode: queue D2H copies of the packets just recovered.
    void download_recovered();

private:
    // ---- window (reference DecoderPacketWindow) ----
    DecSlot& slot(unsigned e) { return subwindows_[e / kSubwindow]->slot[e % kSubwindow]; }
    unsigned column_to_element(unsigned c) const { return column_sub(c, columnStart_); }
    unsigned element_to_column(unsigned e) const { return column_add(e, columnStart_); }
    unsigned next_lane_element(unsigned element, unsigned lane) const
    {
        unsigned e = element - (element % kLanes) + lane;
        return e < element ? e + kLanes : e;
    }
    bool mark_got(unsigned column);
    /// A destination for a symbol of `need` bytes in element's slot: its slab
    /// slot or a buffer of its own (false: arena failure).
    bool place(unsigned element, unsigned need);
    void release_slot(DecSlot& s)
    {
        if (!s.inSlab)
            eng_->release(s.buf);
        s.buf = DevBuf();
        s.inSlab = false;
    }
    /// add_original after validation and the duplicate checks: the element's
    /// slot takes its destination (the caller queues the ingest).
    SiameseResult accept_original(unsigned element, unsigned column, unsigned header, unsigned dataBytes);
    unsigned range_lost(unsigned start, unsigned end);
    unsigned find_next_lost(unsigned start);
    unsigned find_next_got(unsigned start);
    void iterate_next_expected(unsigned start);
    bool grow_window(unsigned end);

    struct Sum
    {
        unsigned elementStart = 0, elementEnd = 0;
        DevSum d;
    };
    Sum& sum(unsigned lane, unsigned s) { return lanes_[lane][s]; }
    bool grow_sum(DevSum& s, unsigned bytes);
    void materialize(unsigned lane, unsigned s);
    void cover(unsigned lo, unsigned hi);   // row batch window covers [lo, hi)
    unsigned windowLo_ = 0;                 // lowest element the current row references
    DevSum& get_sum(unsigned lane, unsigned s, unsigned elementEnd);
    /// get_sum's walk of a lane's elements [from, to): valid while the
    /// window's slots are unchanged (scanEpoch_ moves on every change)
    struct LaneScan
    {
        unsigned from = ~0u, to = 0, end = 0, most = 0, got = 0;
        uint64_t epoch = ~0ull;
    };
    LaneScan laneScan_[kLanes];
    uint64_t scanEpoch_ = 0;
    bool start_sums(unsigned elementStart, unsigned bufferBytes);
    void reset_sums(unsigned elementStart);
    bool plug_sum_holes(unsigned elementStart);
    void remove_elements();

    // ---- recovery list (RecoveryPacketList) ----
    void list_insert(RecPacket* r, bool outOfOrder);
    void list_delete_before(unsigned element);
    void free_packet(RecPacket* r);

    // ---- checked region / matrix ----
    void region_reset();
    void matrix_reset();
    bool check_recovery_possible();
    SiameseResult decode_region();
    /// decode()'s search over the checked region (after check_recovery_possible)
    SiameseResult decode_loop(SiameseOriginalPacket** packetsOut, unsigned* countOut);
    /// decode_region after the elimination: its outcome, then the
    /// elimination of received data and the solve
    SiameseResult finish_region(bool solved);
    /// decode_device's two halves
    bool submit_device_ge(bool chained = false);
    SiameseResult finish_device_ge(SiameseOriginalPacket** packetsOut, unsigned* countOut);
    /// The chained form (decode_device): the job, the gated elimination of
    /// received data and the gated solve in one submission; its finish
    bool submit_chained();
    SiameseResult finish_chained(SiameseOriginalPacket** packetsOut, unsigned* countOut);
    unsigned geState_ = 0;               // 1: a device matrix job is queued; 2: a chained one
    unsigned geRows_ = 0, geCols_ = 0;   // ... of this size
    uint32_t geBase_ = 0;                // ... and its first result word
    std::vector<uint32_t> geOut_;        // its output (ops.h GeDesc)
    // the chained decode's deferred accounting (its rows' reference bytes,
    // counted only once the device elimination succeeded) and its solve
    bool deferAccount_ = false;
    uint64_t deferredBytes_ = 0;
    bool chainElimFailed_ = false;       // eliminate_original_data refused (Disabled if the job succeeds)
    unsigned chainSlot_ = 0;             // its solve's Resolver::pend slot
    unsigned chainBytes_ = 0;            // its rows' common length
    void account_elim(uint64_t bytes)
    {
        if (deferAccount_)
            deferredBytes_ += bytes;
        else
            eng_->account(bytes);
    }
    // The decoder's sums as they stood before a chained elimination of
    // received data: restored if the device elimination fails (the gated sum
    // updates did not run), so the host is in the reference's state for the
    // retry.  Sum buffers the elimination replaced are released only once
    // the outcome is known.
    struct SumState
    {
        Sum lanes[kLanes][kSums];
        unsigned columnStart = 0, columnCount = 0;
        std::vector<unsigned> recoveredColumns;
    };
    SumState chainSums_;
    bool deferRelease_ = false;
    std::vector<DevBuf> chainReleases_;
    void release_sum_buf(DevBuf& b)
    {
        if (deferRelease_) {
            chainReleases_.push_back(b);
            b = DevBuf();
        } else {
            eng_->release(b);
        }
    }
    void chain_sums_commit();    // the elimination ran: release what it replaced
    void chain_sums_restore();   // it did not: back to chainSums_
    bool generate_matrix();
    void populate_columns(unsigned oldColumns, unsigned newColumns);
    void populate_rows(unsigned oldRows, unsigned newRows);
    void resume_ge(unsigned oldRows, unsigned rows);
    bool gaussian_elimination();
    bool pivoted_ge(unsigned pivot);
    bool eliminate_row(const uint8_t* geRow, uint8_t* remRow, unsigned pivot, unsigned end,
                       uint8_t valI);
    uint8_t* mrow(unsigned r) { return mat_.data() + (size_t)r * matStride_; }
    bool matrix_resize(unsigned rows, unsigned columns, bool initialize);

    bool eliminate_original_data();
    SiameseResult solve_and_substitute();
    /// solve_and_substitute's halves: the device solve (rows in pivots_
    /// order; gateWord: 1 + the chained job's outcome word, whose solve then
    /// takes the job's coefficients, ops.h GeDesc) and its Resolver slot;
    /// then the host side of BackSubstitution (the window takes the
    /// recovered buffers).  solve_plan returns false on an arena failure.
    bool solve_plan(uint32_t gateWord, unsigned* slotOut);
    SiameseResult solve_publish(unsigned slot);
    SiameseResult publish_final(unsigned slot);   // a chained solve's, its lengths known

    bool add_single(const RowMeta& m, const uint8_t* headBytes, unsigned payloadBytes,
                    const void* hostData, uint64_t devData, Program* producer);
    SiameseResult add_recovery_common(const RowMeta& m, int footerBytes, unsigned totalBytes,
                                      const void* hostData, uint64_t devData,
                                      const uint8_t* headBytes, Program* producer);

    Engine* eng_;
    Program prog_;
    bool mirror_;
    bool disabled_ = false;

    // window
    unsigned count_ = 0;
    unsigned columnStart_ = 0;
    unsigned nextExpected_ = 0;
    std::vector<DecSubwindowPtr> subwindows_;
    Sum lanes_[kLanes][kSums];
    unsigned sumColumnStart_ = 0;
    unsigned sumColumnCount_ = 0;
    std::vector<SiameseOriginalPacket> recovered_;
    bool hasRecovered_ = false;
    std::vector<unsigned> recoveredColumns_;

    // recovery list
    RecPacket* head_ = nullptr;
    RecPacket* tail_ = nullptr;
    unsigned listCount_ = 0;
    RowMeta lastMeta_;
    unsigned lastBytes_ = 0;

    // checked region
    struct
    {
        unsigned elementStart = 0;
        RecPacket* first = nullptr;
        RecPacket* last = nullptr;
        unsigned nextCheckStart = 0;
        unsigned recoveryCount = 0, lostCount = 0;
        bool solveFailed = false;
    } region_;

    // recovery matrix
    struct RowInfo
    {
        RecPacket* rec = nullptr;
        bool used = false;
        unsigned columnCount = 0;
    };
    struct ColInfo
    {
        DecSlot* original = nullptr;
        unsigned column = 0;
    };
    std::vector<RowInfo> rows_;
    std::vector<ColInfo> cols_;
    // per matrix column, for the vector row builder (gf_dense_row): lane,
    // CX and CX^2, each padded by kRowSlack bytes
    static constexpr unsigned kRowSlack = 32;
    std::vector<uint8_t> colLane_, colCx_, colCx2_;
    std::vector<uint32_t> pickCol_;   // generate_matrix: matrix column per element (or none)
    unsigned prevNextCheckStart_ = 0;
    std::vector<uint8_t> mat_;
    unsigned matRows_ = 0, matCols_ = 0, matAllocRows_ = 0, matStride_ = 0;
    std::vector<unsigned> pivots_;
    std::vector<unsigned> geEnd_;   // gaussian_elimination: each pivot row's column count
    unsigned geResume_ = 0;
    // a device elimination came out singular: this decoder's later attempts
    // eliminate on the host, in the round that runs their symbol work (a
    // lone device job is a 48 us latency-bound launch on the step's tail)
    bool geHost_ = false;
    uint64_t geBytes_ = 0;   // coefficient bytes the elimination multiplied (accounting)
    // the current pivot row's bytes after the pivot, split for gf_muladd_prepared
    GfRowSrc geSrc_;
    const uint8_t* geSrcRow_ = nullptr;
    unsigned geSrcPivot_ = 0;

    unsigned latestColumn_ = 0;

    // Recovered slots awaiting their exact length from the device
    struct Fix
    {
        DecSlot* slot;
        uint8_t* buf;          // buffer swapped into the slot by the solve
        uint32_t resultWord;   // column index within the solve's result block
        unsigned outIndex;     // index into recovered_
        unsigned bound;        // upper bound on the length (row length)
    };
    /// A queued solve whose completion has not been applied yet (slots are
    /// reused).  Written by the owner thread when the decode queues the solve
    /// and by the engine's completer thread when its submission completes,
    /// both under Resolver::mu.
    struct PendingDecode
    {
        std::vector<Fix> fixes;       // by descending column: fixes[m - 1 - ci] is column ci
        uint32_t base = 0;
        unsigned m = 0;
        uint64_t serial = 0;
        bool live = false;            // queued, not yet applied to the decoder's slots
        bool done = false;            // the completion arrived: `words` holds the results
        bool held = false;            // a chained solve not yet published (apply_resolved skips it)
        std::vector<uint32_t> words;  // [0] rows recovered, [1 + ci] header << 29 | length
        /// caller-owned outputs to fill at completion (deferred API): (ci, entry)
        std::vector<std::pair<unsigned, SiameseOriginalPacket*>> targets;
    };
    /// Shared between the decoder and the completions it queued, so a freed
    /// decoder never waits for them: a completion that finds the decoder
    /// gone (orphan) still fills the caller-owned entries, nothing else.
    struct Resolver
    {
        std::mutex mu;
        std::vector<PendingDecode> pend;
        std::atomic<uint64_t> doneCount{0};   // completions arrived (monotonic)
        bool orphan = false;
        // the legacy output array (sgpu_decode / siamese_decode, valid until
        // the next decode): patched by the completer when it still belongs to
        // the decode that queued the solve (batch API; the drop-in mirror
        // patches on the owner's thread in apply_resolved)
        SiameseOriginalPacket* out = nullptr;
        size_t outCount = 0;
        uint64_t outSerial = 0;
        bool mirror = false;
        // the output of the decoder's device matrix job (decode_device)
        std::vector<uint32_t> geOut;
        bool geDone = false;
    };
    static void complete_solve(Resolver& r, unsigned slot, const uint32_t* results);
    static void fill_entry(const PendingDecode& pd, unsigned ci, SiameseOriginalPacket& out);
    void apply_resolved();
    void publish_outputs();   // Resolver::out* = recovered_ (caller holds res_->mu)
    std::shared_ptr<Resolver> res_;
    uint64_t appliedCount_ = 0;
    unsigned lastPendSlot_ = 0;   // Resolver::pend slot of the latest queued solve
    std::vector<Fix> lastDecoded_;
    // scratch of solve_and_substitute (reused across decodes)
    std::vector<RecPacket*> scratchRec_;
    std::vector<unsigned> scratchLen_;
    std::vector<SolveRow> scratchRows_;
    std::vector<uint8_t> scratchCoef_;
    uint64_t decodeSerial_ = 0;

    // Heap capacity of the vectors above, handed from a freed decoder to the
    // next one created on the same thread: a bench step creates and frees
    // thousands of decoders, and growing these from empty each time costs
    // ~40 mallocs per decoder on contended heap arenas.
    struct Spare;
    void adopt_spare();
    void donate_spare();
    unsigned pendingSolves_ = 0;

    uint64_t stats_[SiameseDecoderStats_Count] = {};
};

} // namespace sgpu
