// encoder.cpp -- see encoder.h.  Line citations are to the reference
// SiameseEncoder.cpp unless stated otherwise.
#include "encoder.h"

#include <algorithm>
#include <cstring>

namespace sgpu {

EncoderCore::EncoderCore(Engine* eng, bool hostMirror) : eng_(eng), prog_(eng, 0), mirror_(hostMirror)
{
    // Window starts cleared (:63-82)
    for (unsigned l = 0; l < kLanes; ++l)
        for (unsigned s = 0; s < kSums; ++s)
            lanes_[l].next[s] = l;
    // the subwindow table's capacity comes from an encoder freed on this
    // thread (see DecoderCore::Spare)
    if (SubwindowTable* t = CapStash<SubwindowTable>::take()) {
        subwindows_.swap(t->v);
        recoveryHeld_.swap(t->held);
        CapStash<SubwindowTable>::put_shell(t);
    }
}

EncoderCore::~EncoderCore()
{
    // one pass per subwindow: release owned buffers and leave the slots
    // fresh for the pool (EncSubwindowRecycle skips a clean subwindow)
    for (auto& sw : subwindows_) {
        for (EncSlot& s : sw->slot) {
            if (!s.inSlab)
                eng_->release(s.buf);
            s.buf = DevBuf();
            s.inSlab = false;
            s.bytes = s.column = s.header = 0;
            s.lastSend = 0;
            if (s.hostp)
                s.hostp->clear();
        }
        eng_->slab_release(sw->slab);
        sw->slab = Slab();
        sw->clean = true;
    }
    for (Lane& l : lanes_)
        for (DevSum& s : l.sum)
            eng_->release(s.buf);
    eng_->release(recovery_);
    for (DevBuf& b : recoveryHeld_)
        eng_->release(b);
    subwindows_.clear();   // (subwindows go back to their own pool)
    recoveryHeld_.clear();
    SubwindowTable* t = CapStash<SubwindowTable>::shell();
    subwindows_.swap(t->v);
    recoveryHeld_.swap(t->held);
    CapStash<SubwindowTable>::give(t);
}

// ---------------------------------------------------------------------------
// Window bookkeeping

unsigned EncoderCore::take_element()
{
    // :85-161
    const unsigned column = nextColumn_;
    unsigned element = count_;

    // Keep one lane-width of spare slots ahead of the last subwindow (:108-118)
    if (element + kLanes >= subwindows_.size() * kSubwindow) {
        subwindows_.emplace_back(ObjPool<EncSubwindow>::get());
        subwindows_.back()->clean = false;
    }

    if (count_ > 0)
        ++count_;
    else {
        element = column % kLanes;
        start_window(column);
    }
    return element;
}

bool EncoderCore::place(unsigned element, unsigned need)
{
    EncSubwindow* sw = subwindows_[element / kSubwindow].get();
    EncSlot& s = sw->slot[element % kSubwindow];
    release_slot(s);
    bool failed = false;
    s.buf = eng_->slab_slot(sw->slab, element % kSubwindow, need, &failed);
    s.inSlab = (bool)s.buf;
    if (!s.buf && !failed)
        s.buf = eng_->alloc(need);
    if (!s.buf) {
        disabled_ = true;
        return false;
    }
    return true;
}

void EncoderCore::fill_slot(EncSlot& s, unsigned column, unsigned header, unsigned dataBytes, uint32_t stamp)
{
    s.header = header;
    s.bytes = header + dataBytes;
    s.column = column;
    s.lastSend = stamp;

    nextColumn_ = column_add(nextColumn_, 1);

    staleSums_ |= 7u << (column % kLanes * kSums);
    Lane& lane = lanes_[column % kLanes];
    if (lane.longest < s.bytes)
        lane.longest = s.bytes;
    if (longest_ < s.bytes)
        longest_ = s.bytes;

    stats_[SiameseEncoderStats_OriginalCount]++;
    stats_[SiameseEncoderStats_OriginalBytes] += dataBytes;
}

SiameseResult EncoderCore::add(SiameseOriginalPacket& packet, uint64_t deviceSrc)
{
    // :85-161
    if (dead())
        return Siamese_Disabled;
    if (remaining_slots() == 0)
        return Siamese_MaxPacketsReached;

    const unsigned column = nextColumn_;
    packet.PacketNum = column;
    const unsigned element = take_element();

    uint8_t hdr[kMaxLengthPrefix];
    const unsigned h = write_length_prefix(packet.DataBytes, hdr);
    if (!place(element, h + packet.DataBytes))
        return Siamese_Disabled;
    EncSlot& s = slot(element);
    if (deviceSrc)
        prog_.ingest_device(s.buf, deviceSrc, packet.DataBytes, hdr, h);
    else
        prog_.ingest_host(s.buf, packet.Data, packet.DataBytes, hdr, h);
    if (mirror_) {
        s.host().resize(h + packet.DataBytes);
        std::memcpy(s.host().data(), hdr, h);
        std::memcpy(s.host().data() + h, packet.Data, packet.DataBytes);
    }
    fill_slot(s, column, h, packet.DataBytes, (uint32_t)now_msec());
    return Siamese_Success;
}

SiameseResult EncoderCore::add_range(uint64_t src, uint32_t srcStride, const unsigned* lens, unsigned fixedBytes,
                                     unsigned count, unsigned* firstNum, unsigned* added)
{
    *added = 0;
    *firstNum = nextColumn_;
    if (dead())
        return Siamese_Disabled;
    // one timestamp for the call (ARQ's RTO is milliseconds)
    const uint32_t stamp = count ? (uint32_t)now_msec() : 0;
    // the open ingest run: symbols of one length into consecutive slots
    struct
    {
        uint64_t dst = 0, src = 0;
        uint32_t stride = 0, n = 0, bytes = 0, h = 0;
        uint8_t hdr[kMaxLengthPrefix] = {};
    } run;
    auto close_run = [&] {
        if (run.n)
            prog_.ingest_run(run.dst, run.stride, run.src, srcStride, run.n, run.bytes, run.hdr, run.h);
        run.n = 0;
    };
    SiameseResult res = Siamese_Success;
    for (unsigned k = 0; k < count; ++k) {
        const unsigned bytes = lens ? lens[k] : fixedBytes;
        if (bytes == 0 || bytes > SIAMESE_MAX_PACKET_BYTES) {
            res = Siamese_InvalidInput;
            break;
        }
        if (remaining_slots() == 0) {
            res = Siamese_MaxPacketsReached;
            break;
        }
        const unsigned column = nextColumn_;
        const unsigned element = take_element();
        uint8_t hdr[kMaxLengthPrefix];
        const unsigned h = write_length_prefix(bytes, hdr);
        if (!place(element, h + bytes)) {
            res = Siamese_Disabled;
            break;
        }
        EncSlot& s = slot(element);
        const uint64_t from = src + (uint64_t)k * srcStride;
        if (run.n && run.bytes == bytes && run.n < kIngestRunMax && s.buf.cap == run.stride &&
            s.buf.addr() == run.dst + (uint64_t)run.n * run.stride &&
            from == run.src + (uint64_t)run.n * srcStride)
            ++run.n;
        else {
            close_run();
            run.dst = s.buf.addr();
            run.src = from;
            run.stride = s.buf.cap;
            run.n = 1;
            run.bytes = bytes;
            run.h = h;
            std::memcpy(run.hdr, hdr, sizeof(hdr));
        }
        fill_slot(s, column, h, bytes, stamp);
        ++*added;
    }
    close_run();
    return res;
}

void EncoderCore::start_window(unsigned column)
{
    // :163-181 -- element % 8 == column % 8 is an invariant of the window
    const unsigned element = column % kLanes;
    // every element of the old window was acknowledged: slabs start afresh
    for (auto& sw : subwindows_) {
        for (EncSlot& s : sw->slot)
            if (s.inSlab) {
                s.buf = DevBuf();
                s.inSlab = false;
            }
        eng_->slab_release(sw->slab);
    }
    columnStart_ = column - element;
    sumStart_ = element;
    sumEnd_ = element;
    firstUnremoved_ = element;
    count_ = element + 1;
    longest_ = 0;
    for (Lane& l : lanes_)
        l.longest = 0;
    staleSums_ = kAllSums;
    sumTableStale_ = true;
}

void EncoderCore::remove_before(unsigned firstKeptColumn)
{
    // :183-216
    if (dead())
        return;
    const unsigned element = column_to_element(firstKeptColumn);
    if (element >= count_) {
        if (!column_delta_negative(element))
            count_ = 0; // everything acknowledged
        return;
    }
    if (firstUnremoved_ < element)
        firstUnremoved_ = element;
}

void EncoderCore::reset_sums(unsigned elementStart)
{
    // :218-237
    for (unsigned l = 0; l < kLanes; ++l) {
        const unsigned first = next_lane_element(elementStart, l);
        for (unsigned s = 0; s < kSums; ++s) {
            lanes_[l].next[s] = first;
            lanes_[l].sum[s].bytes = 0;
            lanes_[l].sum[s].devValid = 0;
        }
    }
    sumStart_ = elementStart;
    sumEnd_ = elementStart;
    sumColumnStart_ = element_to_column(elementStart);
    sumErased_ = 0;
    staleSums_ = kAllSums;
    sumTableStale_ = true;
}

void EncoderCore::remove_elements()
{
    // :239-357 -- drop whole subwindows before FirstUnremovedElement
    const unsigned keptSub = firstUnremoved_ / kSubwindow;
    const unsigned removed = keptSub * kSubwindow;

    if (sumEnd_ > sumStart_) {
        // Roll the running sums past the removal point before the data goes
        for (unsigned l = 0; l < kLanes; ++l) {
            for (unsigned s = 0; s < kSums; ++s) {
                get_sum(l, s, removed);
                lanes_[l].next[s] -= removed;
            }
        }
        if (removed > sumStart_)
            sumErased_ += removed - sumStart_;
        sumEnd_ = sumEnd_ > removed ? sumEnd_ - removed : 0;
        sumStart_ = sumStart_ > removed ? sumStart_ - removed : 0;
    }

    // window indices shift below: close the open row batch first
    prog_.rows_seal();
    // Removed subwindows rotate to the back for reuse; their slabs go back
    // to the arena (after the flushes that read them)
    for (unsigned i = 0; i < keptSub; ++i) {
        EncSubwindow* sw = subwindows_[i].get();
        for (EncSlot& s : sw->slot)
            if (s.inSlab) {
                s.buf = DevBuf();
                s.inSlab = false;
            }
        eng_->slab_release(sw->slab);
    }
    std::rotate(subwindows_.begin(), subwindows_.begin() + keptSub, subwindows_.end());

    count_ -= removed;
    columnStart_ = element_to_column(removed);
    firstUnremoved_ -= removed;
    staleSums_ = kAllSums;
    sumTableStale_ = true;

    unsigned longest = 0;
    unsigned laneLongest[kLanes] = {0};
    for (unsigned e = firstUnremoved_; e < count_; ++e) {
        const unsigned b = slot(e).bytes;
        longest = std::max(longest, b);
        laneLongest[e % kLanes] = std::max(laneLongest[e % kLanes], b);
    }
    longest_ = longest;
    for (unsigned l = 0; l < kLanes; ++l)
        lanes_[l].longest = laneLongest[l];

    if (sumEnd_ <= sumStart_)
        reset_sums(firstUnremoved_);
}

bool EncoderCore::grow_sum(DevSum& s, unsigned bytes)
{
    if (bytes <= s.bytes)
        return true;
    if (bytes > s.buf.cap) {
        DevBuf nb = eng_->alloc(bytes);
        if (!nb) {
            disabled_ = true;
            return false;
        }
        if (s.devValid) {
            prog_.lc_begin(nb.addr(), s.devValid, 0);
            prog_.lc_term(s.buf.addr(), s.devValid, 1);
            prog_.lc_end();
        }
        eng_->release(s.buf);
        s.buf = nb;
    }
    s.bytes = bytes;
    return true;
}

void EncoderCore::cover(unsigned lo, unsigned hi)
{
    uint32_t from = hi;
    WinEntry* w = prog_.rows_window(lo, hi, &from);
    for (unsigned e = from; e < hi; ++e, ++w) {
        const EncSlot& o = slot(e);
        w->src = o.buf.addr();
        w->len = o.bytes;
        w->column = o.column;
    }
}

DevSum& EncoderCore::get_sum(unsigned lane, unsigned sumIndex, unsigned elementEnd)
{
    // :359-418 -- lazily fold this lane's new originals into the running sum.
    // Sum0 += X, Sum1 += CX*X, Sum2 += CX^2*X.  The terms and coefficients
    // are generated on the device from the row batch's window snapshot.
    Lane& L = lanes_[lane];
    DevSum& sum = L.sum[sumIndex];
    unsigned element = L.next[sumIndex];
    if (element >= elementEnd)
        return sum;

    // The sum grows to the longest original it covers.  L.longest bounds
    // every element of the lane from FirstUnremoved on; older (acknowledged)
    // elements are checked one by one.
    unsigned newBytes = std::max(sum.bytes, L.longest);
    const unsigned end = element + ((elementEnd - element + kLanes - 1) / kLanes) * kLanes;
    for (unsigned e = element; e < end && e < firstUnremoved_; e += kLanes)
        newBytes = std::max(newBytes, slot(e).bytes);
    if (!grow_sum(sum, newBytes))
        return sum;
    // reference source bytes (one add/muladd per original) are counted by
    // the device as it expands the update
    cover(std::min(element, std::min(sumStart_, firstUnremoved_)), end - kLanes + 1);
    prog_.rows_update(lane * kSums + sumIndex, sum.buf.addr(), sum.bytes, sum.devValid, sumIndex,
                      element, end);
    sum.devValid = sum.bytes;
    L.next[sumIndex] = end;
    return sum;
}

SiameseResult EncoderCore::get(SiameseOriginalPacket& packet)
{
    if (dead())
        return Siamese_Disabled;
    const unsigned element = column_to_element(packet.PacketNum);
    if (element >= count_ || slot(element).bytes == 0) {
        packet.Data = nullptr;
        packet.DataBytes = 0;
        return Siamese_NeedMoreData;
    }
    EncSlot& s = slot(element);
    packet.PacketNum = s.column;
    packet.Data = mirror_ ? s.host().data() + s.header : s.buf.ptr + s.header;
    packet.DataBytes = s.bytes - s.header;
    return Siamese_Success;
}

// ---------------------------------------------------------------------------
// Encode

bool EncoderCore::ensure_recovery(unsigned bytes)
{
    for (DevBuf& b : recoveryHeld_)
        eng_->release(b);
    recoveryHeld_.clear();
    // Every recovery packet gets a fresh buffer.  The previous one is
    // recycled only after the flush that produced it completes, so a decoder
    // that copies the packet later in the same flush (its own program, group
    // 1) still reads it intact, and consecutive rows carry no write-after-
    // read dependency through a shared buffer.
    eng_->release(recovery_);
    recovery_ = eng_->alloc(bytes);
    if (!recovery_) {
        disabled_ = true;
        return false;
    }
    return true;
}

void EncoderCore::finish_row(EncodeOut& out, const RowMeta& meta, unsigned payloadBytes,
                             bool footerWritten)
{
    out.meta = meta;
    out.footerBytes = write_footer(meta, out.footer);
    if (!footerWritten)
        prog_.literal(recovery_.addr(), payloadBytes, out.footer, out.footerBytes);
    out.buf = recovery_;
    out.bytes = payloadBytes + out.footerBytes;
    eng_->account(0, out.bytes);
    stats_[SiameseEncoderStats_RecoveryCount]++;
    stats_[SiameseEncoderStats_RecoveryBytes] += out.bytes;
}

SiameseResult EncoderCore::encode(EncodeOut& out)
{
    // :1146-1254
    lastRowSiamese_ = false;
    if (dead())
        return Siamese_Disabled;
    if (count_ == 0) {
        out.bytes = 0;
        return Siamese_NeedMoreData;
    }
    if (firstUnremoved_ >= kRemoveThreshold)
        remove_elements();

    const unsigned inFlight = unacked();
    if (inFlight == 1)
        return single_row(out);

    const unsigned sumWidthBound = count_ - sumStart_ + sumErased_;
    if (sumEnd_ <= sumStart_ || sumWidthBound >= kMaxPacketsInFlight) {
        if (inFlight <= kCauchyThreshold)
            return cauchy_row(out);
        reset_sums(firstUnremoved_);
    } else if (inFlight <= kSumResetThreshold || sumWidthBound <= kCauchyThreshold) {
        sumEnd_ = sumStart_; // stop the running sums
        return cauchy_row(out);
    }

    const unsigned row = nextRow_;
    if (++nextRow_ >= kRowValuePeriod)
        nextRow_ = 0;
    return siamese_row(out, row);
}

SiameseResult EncoderCore::encode_range(EncodeOut* out, unsigned count, unsigned* produced)
{
    for (DevBuf& b : recoveryHeld_)   // (the previous call's packets)
        eng_->release(b);
    recoveryHeld_.clear();
    return encode_range_more(out, count, produced);
}

SiameseResult EncoderCore::encode_range_more(EncodeOut* out, unsigned count, unsigned* produced)
{
    *produced = 0;
    std::vector<DevBuf> held;   // this call's packets before the last (and the chunks' before it)
    held.swap(recoveryHeld_);   // (capacity reused; ensure_recovery below finds none to release)
    SiameseResult r = Siamese_Success;
    // After a Siamese row, encode() would choose a Siamese row again: its
    // path depends on the window only, which no call of a range changes.
    // Those rows skip the per-call dispatch and share one accounting.
    bool siamese = false;
    uint64_t opAcc = 0, outAcc = 0;
    for (unsigned k = 0; k < count; ++k) {
        if (k > 0 || !held.empty() || *produced) {
            // keep the previous packet: ensure_recovery would release it
            held.push_back(recovery_);
            recovery_ = DevBuf();
        }
        if (siamese) {
            if (dead()) {
                r = Siamese_Disabled;
                break;
            }
            const unsigned row = nextRow_;
            if (++nextRow_ >= kRowValuePeriod)
                nextRow_ = 0;
            recovery_ = eng_->alloc(longest_ + kMaxFooterBytes);
            if (!recovery_) {
                disabled_ = true;
                r = Siamese_Disabled;
                break;
            }
            uint64_t ob = 0;
            r = siamese_row_body(out[k], row, &ob);
            if (r != Siamese_Success)
                break;
            opAcc += ob;
            outAcc += out[k].bytes;
        } else {
            r = encode(out[k]);
            if (r != Siamese_Success)
                break;
            siamese = lastRowSiamese_;
        }
        ++*produced;
    }
    eng_->account(opAcc, outAcc);
    recoveryHeld_.swap(held);
    return r;
}

SiameseResult EncoderCore::single_row(EncodeOut& out)
{
    // :1296-1329 -- the lone original itself, with a SumCount=1 footer
    const EncSlot& o = slot(firstUnremoved_);
    if (!ensure_recovery(o.bytes + kMaxFooterBytes))
        return Siamese_Disabled;
    prog_.lc_begin(recovery_.addr(), o.bytes, 0);
    prog_.lc_term(o.buf.addr(), o.bytes, 1);
    prog_.lc_end();
    write_length_prefix(o.bytes - o.header, out.head);
    RowMeta m;
    m.sumCount = 1;
    m.ldpcCount = 1;
    m.columnStart = o.column;
    m.row = 0;
    finish_row(out, m, o.bytes);
    return Siamese_Success;
}

SiameseResult EncoderCore::cauchy_row(EncodeOut& out)
{
    // :1334-1441 -- parity row (Row 0) or Cauchy row over the unacked window
    const unsigned first = firstUnremoved_;
    if (!ensure_recovery(longest_ + kMaxFooterBytes))
        return Siamese_Disabled;
    const unsigned inFlight = unacked();
    RowMeta m;
    m.sumCount = inFlight;
    m.ldpcCount = inFlight;
    m.columnStart = element_to_column(first);

    unsigned used = 0;
    for (unsigned e = first; e < count_; ++e)
        used = std::max(used, slot(e).bytes);
    prog_.lc_begin(recovery_.addr(), used, 0);
    uint64_t opBytes = 0;

    const unsigned parityElement = column_to_element(nextParityColumn_);
    if (parityElement <= first || column_delta_negative(parityElement)) {
        nextParityColumn_ = column_add(m.columnStart, inFlight);
        m.row = 0;
        for (unsigned e = first; e < count_; ++e) {
            const EncSlot& o = slot(e);
            prog_.lc_term(o.buf.addr(), o.bytes, 1);
            // the reference memcpy's the first parity column (no GF op)
            if (e > first)
                opBytes += o.bytes;
        }
    } else {
        const unsigned crow = nextCauchyRow_;
        m.row = crow + 1;
        if (++nextCauchyRow_ >= kCauchyMaxRows)
            nextCauchyRow_ = 0;
        unsigned ccol = m.columnStart % kCauchyMaxColumns;
        for (unsigned e = first; e < count_; ++e) {
            const EncSlot& o = slot(e);
            prog_.lc_term(o.buf.addr(), o.bytes, cauchy_element(crow, ccol));
            opBytes += o.bytes;
            ccol = (ccol + 1) % kCauchyMaxColumns;
        }
    }
    prog_.lc_end();
    eng_->account(opBytes);
    finish_row(out, m, used);
    return Siamese_Success;
}

SiameseResult EncoderCore::siamese_row(EncodeOut& out, unsigned row)
{
    if (!ensure_recovery(longest_ + kMaxFooterBytes))
        return Siamese_Disabled;
    uint64_t opBytes = 0;
    const SiameseResult r = siamese_row_body(out, row, &opBytes);
    if (r == Siamese_Success)
        eng_->account(opBytes, out.bytes);
    return r;
}

SiameseResult EncoderCore::siamese_row_body(EncodeOut& out, unsigned row, uint64_t* opBytesOut)
{
    const unsigned recoveryBytes = longest_;

    // Dense part (:1046-1098): opcode bits 0-2 feed the row, 3-5 the product.
    // The lane sums are brought up to date first (their own ops precede the
    // row in the program); the row selects them by mask bit lane*3 + sum.
    // Only sums that may have fallen behind since they were last folded
    // (staleSums_) are visited, so consecutive rows over an unchanged window
    // skip the lazy-update walk.
    const RowSelect& sel = row_select(row);
    const uint32_t want = sel.mask[0] | sel.mask[1];
    uint32_t need = want & staleSums_;
    if (need)
        sumTableStale_ = true;   // a sum may grow below
    for (; need; need &= need - 1) {
        const unsigned k = (unsigned)__builtin_ctz(need);
        get_sum(k / kSums, k % kSums, count_);
        if (dead())
            return Siamese_Disabled;
    }
    staleSums_ &= ~want;
    if (sumTableStale_ || sumClipBytes_ != recoveryBytes) {
        // the 24 sums as the rows read them (rebuilt only after a change),
        // and the reference source bytes of each (clipped to the row)
        sumTableStale_ = false;
        sumTableVersion_ = Program::next_table_version();
        sumPresent_ = 0;
        sumClipBytes_ = recoveryBytes;
        for (unsigned k = 0; k < kRowSums; ++k) {
            const DevSum& d = lanes_[k / kSums].sum[k % kSums];
            WinEntry& t = sumTable_[k];
            t.src = d.buf.addr();
            t.len = d.bytes;
            t.column = 0;
            if (d.bytes > 0)
                sumPresent_ |= 1u << k;
            sumClip_[k] = std::min(d.bytes, recoveryBytes);
        }
    }
    const uint32_t mask[2] = {sel.mask[0] & sumPresent_, sel.mask[1] & sumPresent_};
    uint64_t opBytes = recoveryBytes; // final RX * product muladd
    for (unsigned h = 0; h < 2; ++h)
        for (uint32_t b = mask[h]; b; b &= b - 1)
            opBytes += sumClip_[__builtin_ctz(b)];
    sumEnd_ = count_;

    RowMeta m;
    m.sumCount = sumEnd_ - sumStart_ + sumErased_;
    m.ldpcCount = unacked();
    m.columnStart = sumColumnStart_;
    m.row = row;
    const unsigned footerBytes = write_footer(m, out.footer);

    // Sparse part (:1100-1144): ceil(n/16) PCG-chosen pairs, drawn on the
    // device, which also counts their reference source bytes
    const unsigned start = firstUnremoved_;
    const unsigned n = sumEnd_ - start;

    // Recovery = row sums ^ RX * product (:1232-1233) and its footer: one row
    // of the program's Siamese row batch (consecutive rows share the sums)
    cover(std::min(start, sumStart_), sumEnd_);
    prog_.rows_row(sumTable_, recovery_.addr(), recoveryBytes, 0, row_value(row), mask[0], mask[1], row,
                   n, start, count_, out.footer, footerBytes, sumTableVersion_);

    out.meta = m;
    out.footerBytes = footerBytes;
    out.buf = recovery_;
    out.bytes = recoveryBytes + footerBytes;
    stats_[SiameseEncoderStats_RecoveryCount]++;
    stats_[SiameseEncoderStats_RecoveryBytes] += out.bytes;
    lastRowSiamese_ = true;
    *opBytesOut = opBytes;
    return Siamese_Success;
}

SiameseResult EncoderCore::stats(uint64_t* out, unsigned count)
{
    if (count > SiameseEncoderStats_Count)
        count = SiameseEncoderStats_Count;
    uint64_t mem = recovery_.cap;
    for (auto& sw : subwindows_) {
        mem += sw->slab.buf.cap;
        for (EncSlot& s : sw->slot)
            if (!s.inSlab)
                mem += s.buf.cap;
    }
    for (Lane& l : lanes_)
        for (DevSum& s : l.sum)
            mem += s.buf.cap;
    stats_[SiameseEncoderStats_MemoryUsed] = mem;
    for (unsigned i = 0; i < count; ++i)
        out[i] = stats_[i];
    return Siamese_Success;
}

} // namespace sgpu
