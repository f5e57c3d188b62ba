// encoder.h -- host control plane of the encoder.
//
// Decision logic (window bookkeeping, path selection, row numbering, footer)
// follows the reference encoder exactly so the emitted bit stream is
// identical (reference SiameseEncoder.h:104-421, SiameseEncoder.cpp:56-1441).
// Every symbol-sized operation is emitted as a device op into this
// instance's Program; the symbols themselves live in HBM.
#pragma once

#include "arq.h"
#include "codedef.h"
#include "engine.h"
#include "objpool.h"
#include "../../include/siamese.h"

#include <memory>
#include <vector>

namespace sgpu {

struct EncSlot
{
    DevBuf buf;                 // [length prefix || payload] in HBM
    bool inSlab = false;        // buf is a slot of the subwindow's slab (not owned)
    unsigned bytes = 0;         // prefix + payload
    unsigned column = 0;
    unsigned header = 0;        // length-prefix bytes
    uint32_t lastSend = 0;      // msec timestamp of the last (re)send (ARQ)
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

struct EncSubwindow
{
    EncSlot slot[kSubwindow];
    Slab slab;                  // the slots' shared buffer (engine.h)
    bool clean = false;         // every slot already in its fresh state (the owner's teardown)
};

/// unique_ptr deleter: subwindows go back to the thread's pool, emptied
/// (their buffers were released by the owner).
struct EncSubwindowRecycle
{
    void operator()(EncSubwindow* w) const
    {
        if (!w->clean) {
            w->slab = Slab();
            for (EncSlot& s : w->slot) {
                s.buf = DevBuf();
                s.inSlab = false;
                s.bytes = s.column = s.header = 0;
                s.lastSend = 0;
                if (s.hostp)
                    s.hostp->clear();
            }
            w->clean = true;
        }
        ObjPool<EncSubwindow>::put(w);
    }
};
using EncSubwindowPtr = std::unique_ptr<EncSubwindow, EncSubwindowRecycle>;

/// Running sum of one (lane, sum-index) in HBM.
struct DevSum
{
    DevBuf buf;
    unsigned bytes = 0;     // logical length (reference Buffer.Bytes)
    unsigned devValid = 0;  // bytes actually materialised on the device
};

/// Result of an encode in device terms.
struct EncodeOut
{
    DevBuf buf;             // recovery packet (valid until the next encode)
    unsigned bytes = 0;     // payload + footer
    uint8_t footer[kMaxFooterBytes] = {};
    unsigned footerBytes = 0;
    uint8_t head[kMaxLengthPrefix] = {}; // first bytes (single-packet rows only)
    RowMeta meta;
};

class EncoderCore
{
public:
    EncoderCore(Engine* eng, bool hostMirror);
    ~EncoderCore();

    Program& program() { return prog_; }

    unsigned remaining_slots() const { return kMaxPacketsInFlight - count_; }

    /// siamese_encoder_add.  Source is host memory or (device != 0) HBM.
    SiameseResult add(SiameseOriginalPacket& packet, uint64_t deviceSrc = 0);
    /// `count` adds of device originals in one call (sgpu_encoder_add_range):
    /// original k at src + k * srcStride, lens[k] bytes (fixedBytes when lens
    /// is null).  Identical to `count` add() calls that stop at the first
    /// failure, whose result is returned; *added originals were taken, the
    /// first as packet *firstNum (the rest follow it).  Consecutive slab slots
    /// become one ingest run.
    SiameseResult add_range(uint64_t src, uint32_t srcStride, const unsigned* lens, unsigned fixedBytes,
                            unsigned count, unsigned* firstNum, unsigned* added);
    void remove_before(unsigned firstKeptColumn);
    SiameseResult get(SiameseOriginalPacket& packet);
    /// Generate the next recovery packet (device ops queued, not flushed).
    SiameseResult encode(EncodeOut& out);
    /// `count` encode() calls in one (sgpu_encode_range): out[k] as the k-th
    /// call fills it, stopping at the first call that does not succeed (its
    /// result returned, Success otherwise); *produced = packets made.  Every
    /// packet's buffer stays valid until the next encode call.
    SiameseResult encode_range(EncodeOut* out, unsigned count, unsigned* produced);
    /// encode_range continued: the packets of the call before are kept too
    /// (one sgpu_encode_range made in several chunks).
    SiameseResult encode_range_more(EncodeOut* out, unsigned count, unsigned* produced);
    SiameseResult stats(uint64_t* out, unsigned count);
    /// ARQ: siamese_encoder_ack / siamese_encoder_retransmit (arq.cpp)
    SiameseResult acknowledge(const uint8_t* data, unsigned bytes, unsigned& nextExpectedOut);
    SiameseResult retransmit(SiameseOriginalPacket& out);

    /// Disabled: this instance failed (sticky), or the device did (Engine::failed).
    bool disabled() const { return dead(); }
    bool dead() const { return disabled_ || eng_->failed(); }
    uint64_t stat(unsigned i) const { return stats_[i]; }

private:
    // window (reference EncoderPacketWindow)
    EncSlot& slot(unsigned element)
    {
        return subwindows_[element / kSubwindow]->slot[element % kSubwindow];
    }
    unsigned column_to_element(unsigned c) const { return column_sub(c, columnStart_); }
    unsigned element_to_column(unsigned e) const { return column_add(e, columnStart_); }
    unsigned next_lane_element(unsigned element, unsigned lane) const
    {
        unsigned e = element - (element % kLanes) + lane;
        return e < element ? e + kLanes : e;
    }
    unsigned unacked() const { return count_ - firstUnremoved_; }
    /// The window bookkeeping of one add (reference :85-161) up to its slot:
    /// the element the packet takes (its column is nextColumn_ before).
    unsigned take_element();
    /// Give element's slot a destination for `need` bytes: its slab slot, or
    /// a buffer of its own.  False on an arena failure (the encoder is then
    /// disabled).
    bool place(unsigned element, unsigned need);
    /// The slot's fields and the window's lengths after its symbol is queued.
    void fill_slot(EncSlot& s, unsigned column, unsigned header, unsigned dataBytes, uint32_t stamp);
    void release_slot(EncSlot& s)
    {
        if (!s.inSlab)
            eng_->release(s.buf);
        s.buf = DevBuf();
        s.inSlab = false;
    }
    void start_window(unsigned column);
    void reset_sums(unsigned elementStart);
    void remove_elements();
    /// Lazily accumulate lane sums up to elementEnd; returns the sum.
    DevSum& get_sum(unsigned lane, unsigned sumIndex, unsigned elementEnd);
    void cover(unsigned lo, unsigned hi);   // row batch window covers [lo, hi)
    bool grow_sum(DevSum& s, unsigned bytes);

    SiameseResult single_row(EncodeOut& out);
    SiameseResult cauchy_row(EncodeOut& out);
    SiameseResult siamese_row(EncodeOut& out, unsigned row);
    /// siamese_row without the buffer (recovery_ holds it) and the
    /// accounting (*opBytes: the row's reference source bytes)
    SiameseResult siamese_row_body(EncodeOut& out, unsigned row, uint64_t* opBytes);
    bool ensure_recovery(unsigned bytes);
    void finish_row(EncodeOut& out, const RowMeta& meta, unsigned payloadBytes,
                    bool footerWritten = false);
    void update_rto();
    SiameseResult retransmit_slot(EncSlot& s, SiameseOriginalPacket& out);
    AckState ack_;

    Engine* eng_;
    Program prog_;
    bool mirror_;
    bool disabled_ = false;

    std::vector<EncSubwindowPtr> subwindows_;
    struct SubwindowTable
    {
        std::vector<EncSubwindowPtr> v;
        std::vector<DevBuf> held;   // (recoveryHeld_'s capacity)
    };
    unsigned nextColumn_ = 0;
    unsigned count_ = 0;
    unsigned columnStart_ = 0;
    unsigned longest_ = 0;
    unsigned firstUnremoved_ = 0;
    unsigned sumStart_ = 0, sumEnd_ = 0, sumColumnStart_ = 0, sumErased_ = 0;

    struct Lane
    {
        unsigned next[kSums];
        DevSum sum[kSums];
        unsigned longest = 0;
    } lanes_[kLanes];

    // sums (bit lane*3 + s) that may lag the window: set when an original
    // lands in their lane or the sums restart, cleared once a row folds them
    static constexpr uint32_t kAllSums = (1u << kRowSums) - 1;
    uint32_t staleSums_ = kAllSums;
    // the sums as rows read them (WinEntry per bit), valid unless stale
    WinEntry sumTable_[kRowSums];
    uint32_t sumPresent_ = 0;   // sums holding bytes
    bool sumTableStale_ = true;
    uint64_t sumTableVersion_ = 0;   // Program::rows_row's tag of sumTable_ as last rebuilt
    uint32_t sumClip_[kRowSums] = {};   // min(sum bytes, sumClipBytes_): reference source bytes
    unsigned sumClipBytes_ = ~0u;       // the row length sumClip_ was made for
    bool lastRowSiamese_ = false;       // the last encode() made a Siamese row

    DevBuf recovery_;          // reused recovery packet buffer
    std::vector<DevBuf> recoveryHeld_;   // encode_range's earlier packets (released by the next encode)
    unsigned nextRow_ = 0;
    unsigned nextParityColumn_ = 0;
    unsigned nextCauchyRow_ = 0;

    uint64_t stats_[SiameseEncoderStats_Count] = {};
};

} // namespace sgpu
