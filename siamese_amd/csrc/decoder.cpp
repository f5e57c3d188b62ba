// decoder.cpp -- see decoder.h.  Line citations are to the reference
// SiameseDecoder.cpp unless stated otherwise.
#include "decoder.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <x86intrin.h>

namespace sgpu {

namespace {

inline unsigned popcount_range(uint64_t bits, unsigned begin, unsigned end)
{
    if (begin >= end)
        return 0;
    uint64_t mask = (end >= 64 ? ~0ULL : ((1ULL << end) - 1)) & ~((1ULL << begin) - 1);
    return (unsigned)__builtin_popcountll(bits & mask);
}

inline unsigned first_clear(uint64_t bits, unsigned from)
{
    if (from >= 64)
        return 64;
    const uint64_t inv = ~bits & (~0ULL << from);
    return inv ? (unsigned)__builtin_ctzll(inv) : 64;
}

} // namespace

DecoderCore::DecoderCore(Engine* eng, bool hostMirror)
    : eng_(eng), prog_(eng, 1), mirror_(hostMirror)
{
    adopt_spare();
    if (!res_)
        res_ = std::make_shared<Resolver>();
    res_->mirror = mirror_;
}

// Every recycled vector is empty in a fresh decoder; a spare holds them
// cleared (capacity kept), so swapping one in leaves the decoder in exactly
// its freshly constructed state.  The resolver is recycled only when no
// completion holds it any more (its slots all idle; a slot is claimed by the
// first search for a non-live one and fully rewritten).
struct DecoderCore::Spare
{
    std::vector<DecSubwindowPtr> subwindows;
    std::vector<SiameseOriginalPacket> recovered;
    std::vector<unsigned> recoveredColumns;
    std::vector<RowInfo> rows;
    std::vector<ColInfo> cols;
    std::vector<uint8_t> colLane, colCx, colCx2;
    std::vector<uint32_t> pickCol;
    std::vector<uint8_t> mat;
    std::vector<unsigned> pivots;
    std::shared_ptr<Resolver> res;
    std::vector<Fix> lastDecoded;
    std::vector<RecPacket*> scratchRec;
    std::vector<unsigned> scratchLen;
    std::vector<SolveRow> scratchRows;
    std::vector<uint8_t> scratchCoef;
    std::vector<unsigned> geEnd;
    std::vector<DevBuf> chainReleases;
    std::vector<unsigned> chainColumns;   // (chainSums_.recoveredColumns)
    std::vector<uint32_t> geOut;
};

void DecoderCore::adopt_spare()
{
    Spare* s = CapStash<Spare>::take();
    if (!s)
        return;
    subwindows_.swap(s->subwindows);
    recovered_.swap(s->recovered);
    recoveredColumns_.swap(s->recoveredColumns);
    rows_.swap(s->rows);
    cols_.swap(s->cols);
    colLane_.swap(s->colLane);
    colCx_.swap(s->colCx);
    colCx2_.swap(s->colCx2);
    pickCol_.swap(s->pickCol);
    mat_.swap(s->mat);
    pivots_.swap(s->pivots);
    res_.swap(s->res);
    lastDecoded_.swap(s->lastDecoded);
    scratchRec_.swap(s->scratchRec);
    scratchLen_.swap(s->scratchLen);
    scratchRows_.swap(s->scratchRows);
    scratchCoef_.swap(s->scratchCoef);
    geEnd_.swap(s->geEnd);
    chainReleases_.swap(s->chainReleases);
    chainSums_.recoveredColumns.swap(s->chainColumns);
    geOut_.swap(s->geOut);
    CapStash<Spare>::put_shell(s);   // (now holding this decoder's empty vectors)
}

void DecoderCore::donate_spare()
{
    Spare* s = CapStash<Spare>::shell();
    subwindows_.clear();   // (subwindows go back to their own pool)
    recovered_.clear();
    recoveredColumns_.clear();
    rows_.clear();
    cols_.clear();
    colLane_.clear();
    colCx_.clear();
    colCx2_.clear();
    pickCol_.clear();
    // (mat_ keeps its size: generate_matrix writes every byte of a fresh
    // matrix it reads, so the next decoder skips a zero fill of the bytes)
    pivots_.clear();
    if (res_ && res_.use_count() == 1) {
        // no completion holds it: back to its freshly constructed state
        for (PendingDecode& pd : res_->pend) {
            pd.fixes.clear();
            pd.words.clear();
            pd.targets.clear();
            pd.base = 0;
            pd.m = 0;
            pd.serial = 0;
            pd.live = false;
            pd.done = false;
            pd.held = false;
        }
        res_->doneCount.store(0, std::memory_order_relaxed);
        res_->orphan = false;
        res_->out = nullptr;
        res_->outCount = 0;
        res_->outSerial = 0;
        res_->geOut.clear();
        res_->geDone = false;
    } else if (res_) {
        // completions still queued or in flight: they fill the caller-owned
        // entries they carry and leave this decoder's memory alone
        std::lock_guard<std::mutex> g(res_->mu);
        res_->orphan = true;
        res_->out = nullptr;
        res_->outCount = 0;
        res_.reset();
    }
    lastDecoded_.clear();
    scratchRec_.clear();
    scratchLen_.clear();
    scratchRows_.clear();
    scratchCoef_.clear();
    geEnd_.clear();
    chainReleases_.clear();
    chainSums_.recoveredColumns.clear();
    geOut_.clear();
    subwindows_.swap(s->subwindows);
    recovered_.swap(s->recovered);
    recoveredColumns_.swap(s->recoveredColumns);
    rows_.swap(s->rows);
    cols_.swap(s->cols);
    colLane_.swap(s->colLane);
    colCx_.swap(s->colCx);
    colCx2_.swap(s->colCx2);
    pickCol_.swap(s->pickCol);
    mat_.swap(s->mat);
    pivots_.swap(s->pivots);
    res_.swap(s->res);
    lastDecoded_.swap(s->lastDecoded);
    scratchRec_.swap(s->scratchRec);
    scratchLen_.swap(s->scratchLen);
    scratchRows_.swap(s->scratchRows);
    scratchCoef_.swap(s->scratchCoef);
    geEnd_.swap(s->geEnd);
    chainReleases_.swap(s->chainReleases);
    chainSums_.recoveredColumns.swap(s->chainColumns);
    geOut_.swap(s->geOut);
    CapStash<Spare>::give(s);
}

DecoderCore::~DecoderCore()
{
    // (completions still queued or in flight hold the shared resolver, not
    // this decoder: nothing to wait for, see donate_spare)
    for (RecPacket* r = head_; r;) {
        RecPacket* n = r->next;
        free_packet(r);
        r = n;
    }
    // one pass over each subwindow: release the buffers slots own and leave
    // every slot fresh, so the pool's recycle (DecSubwindowRecycle) need not
    // walk them again (a decoder's teardown is memory-bound on these slots)
    for (auto& sw : subwindows_) {
        for (DecSlot& s : sw->slot) {
            if (!s.inSlab)
                eng_->release(s.buf);
            s.buf = DevBuf();
            s.inSlab = false;
            s.bytes = 0;
            s.column = 0;
            s.header = 0;
            s.pending = false;
            if (s.hostp)
                s.hostp->clear();
        }
        sw->got = 0;
        sw->gotCount = 0;
        eng_->slab_release(sw->slab);
        sw->slab = Slab();
        sw->clean = true;
    }
    for (auto& lane : lanes_)
        for (Sum& s : lane)
            eng_->release(s.d.buf);
    if (geState_ == 2)
        chain_sums_commit();   // (a chained decode never finished: its replaced sum buffers)
    donate_spare();
}

// ---------------------------------------------------------------------------
// Receive window (:1260-1536)

bool DecoderCore::mark_got(unsigned column)
{
    const unsigned element = column_to_element(column);
    if (element >= count_) {
        disabled_ = true;
        return false;
    }
    DecSubwindow* sw = subwindows_[element / kSubwindow].get();
    sw->gotCount++;
    sw->got |= 1ULL << (element % kSubwindow);
    return element == nextExpected_;
}

unsigned DecoderCore::range_lost(unsigned start, unsigned end)
{
    if (start >= end)
        return 0;
    unsigned lost = 0;
    unsigned sub = start / kSubwindow;
    const unsigned bitStart = start % kSubwindow;
    if (bitStart > 0) {
        unsigned bitEnd = bitStart + end - start;
        if (bitEnd > kSubwindow)
            bitEnd = kSubwindow;
        lost += (bitEnd - bitStart) - popcount_range(subwindows_[sub]->got, bitStart, bitEnd);
        ++sub;
    }
    const unsigned subEnd = end / kSubwindow;
    for (unsigned i = sub; i < subEnd; ++i)
        lost += kSubwindow - subwindows_[i]->gotCount;
    if (subEnd >= sub) {
        const unsigned lastBits = end - subEnd * kSubwindow;
        if (lastBits > 0)
            lost += lastBits - popcount_range(subwindows_[subEnd]->got, 0, lastBits);
    }
    return lost;
}

unsigned DecoderCore::find_next_lost(unsigned start)
{
    if (start >= count_)
        return count_;
    const unsigned subEnd = (count_ + kSubwindow - 1) / kSubwindow;
    unsigned sub = start / kSubwindow;
    unsigned bit = start % kSubwindow;
    while (sub < subEnd) {
        const DecSubwindow* sw = subwindows_[sub].get();
        if (sw->gotCount < kSubwindow) {
            bit = first_clear(sw->got, bit);
            if (bit < kSubwindow) {
                const unsigned e = sub * kSubwindow + bit;
                return e > count_ ? count_ : e;
            }
        }
        bit = 0;
        ++sub;
    }
    return count_;
}

void DecoderCore::iterate_next_expected(unsigned start)
{
    if (nextExpected_ >= count_)
        return;
    nextExpected_ = find_next_lost(start);
}

bool DecoderCore::grow_window(unsigned end)
{
    const unsigned needed = (end + kLanes + kSubwindow - 1) / kSubwindow;
    while (subwindows_.size() < needed) {
        subwindows_.emplace_back(ObjPool<DecSubwindow>::get());
        subwindows_.back()->clean = false;
    }
    if (end > count_)
        count_ = end;
    return true;
}

bool DecoderCore::place(unsigned element, unsigned need)
{
    DecSubwindow* sw = subwindows_[element / kSubwindow].get();
    DecSlot& s = sw->slot[element % kSubwindow];
    release_slot(s);
    bool failed = false;
    s.buf = eng_->slab_slot(sw->slab, element % kSubwindow, need, &failed);
    s.inSlab = (bool)s.buf;
    if (!s.buf && !failed)
        s.buf = eng_->alloc(need);
    return (bool)s.buf;
}

SiameseResult DecoderCore::accept_original(unsigned element, unsigned column, unsigned header, unsigned dataBytes)
{
    if (!place(element, header + dataBytes)) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    DecSubwindow* sw = subwindows_[element / kSubwindow].get();
    const unsigned bit = element % kSubwindow;
    DecSlot& s = sw->slot[bit];
    s.header = header;
    s.bytes = header + dataBytes;
    s.column = column;
    s.pending = false;

    sw->gotCount++;
    sw->got |= 1ULL << bit;

    if (element == nextExpected_) {
        iterate_next_expected(element + 1);
        list_delete_before(nextExpected_);
    }
    if (element >= region_.elementStart && element < region_.nextCheckStart)
        region_reset();

    stats_[SiameseDecoderStats_OriginalCount]++;
    stats_[SiameseDecoderStats_OriginalBytes] += dataBytes;
    return Siamese_Success;
}

SiameseResult DecoderCore::add_original(const SiameseOriginalPacket& packet, uint64_t deviceSrc)
{
    settle();
    // :1467-1536
    if (dead())
        return Siamese_Disabled;
    const unsigned element = column_to_element(packet.PacketNum);
    if (column_delta_negative(element)) {
        stats_[SiameseDecoderStats_DupedOriginalCount]++;
        return Siamese_DuplicateData;
    }
    grow_window(element + 1);
    DecSlot& s = slot(element);
    if (s.bytes > 0) {
        stats_[SiameseDecoderStats_DupedOriginalCount]++;
        return Siamese_DuplicateData;
    }

    uint8_t hdr[kMaxLengthPrefix];
    const unsigned h = write_length_prefix(packet.DataBytes, hdr);
    // (the slot keeps its place across the bookkeeping: subwindows_ only grows above)
    const SiameseResult r = accept_original(element, packet.PacketNum, h, packet.DataBytes);
    if (r != Siamese_Success)
        return r;
    if (deviceSrc)
        prog_.ingest_device(s.buf, deviceSrc, packet.DataBytes, hdr, h);
    else
        prog_.ingest_host(s.buf, packet.Data, packet.DataBytes, hdr, h);
    if (mirror_) {
        s.host().resize(h + packet.DataBytes);
        std::memcpy(s.host().data(), hdr, h);
        std::memcpy(s.host().data() + h, packet.Data, packet.DataBytes);
    }
    return Siamese_Success;
}

SiameseResult DecoderCore::add_original_range(unsigned firstNum, uint64_t src, uint32_t srcStride,
                                              const unsigned* lens, unsigned fixedBytes, unsigned count,
                                              SiameseResult* results, unsigned* added)
{
    *added = 0;
    settle();
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
        const unsigned num = (firstNum + k) & SIAMESE_PACKET_NUM_MAX;
        const unsigned bytes = lens ? lens[k] : fixedBytes;
        SiameseResult r = Siamese_Success;
        const unsigned element = column_to_element(num);
        if (bytes == 0 || bytes > SIAMESE_MAX_PACKET_BYTES)
            r = Siamese_InvalidInput;
        else if (dead())
            r = Siamese_Disabled;
        else if (column_delta_negative(element))
            r = Siamese_DuplicateData;
        else {
            grow_window(element + 1);
            if (slot(element).bytes > 0)
                r = Siamese_DuplicateData;
        }
        if (r == Siamese_DuplicateData)
            stats_[SiameseDecoderStats_DupedOriginalCount]++;
        if (r == Siamese_Success) {
            uint8_t hdr[kMaxLengthPrefix];
            const unsigned h = write_length_prefix(bytes, hdr);
            r = accept_original(element, num, h, bytes);
            if (r == Siamese_Success) {
                const DecSlot& s = slot(element);
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
            }
        }
        if (results)
            results[k] = r;
        ++*added;
        if (r != Siamese_Success && r != Siamese_DuplicateData) {
            res = r;
            break;
        }
    }
    close_run();
    return res;
}

// ---------------------------------------------------------------------------
// Running sums over received originals (:1538-1739)

bool DecoderCore::grow_sum(DevSum& s, unsigned bytes)
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
        release_sum_buf(s.buf);
        s.buf = nb;
    }
    s.bytes = bytes; // [devValid, bytes) is zero, materialised lazily
    return true;
}

void DecoderCore::cover(unsigned lo, unsigned hi)
{
    uint32_t from = hi;
    WinEntry* w = prog_.rows_window(lo, hi, &from);
    for (unsigned e = from; e < hi; ++e, ++w) {
        const DecSlot& o = slot(e);
        // lost originals read as absent (their `column` is a matrix column)
        w->src = o.bytes ? o.buf.addr() : 0;
        w->len = o.bytes;
        w->column = o.bytes ? o.column : 0;
    }
}

void DecoderCore::materialize(unsigned lane, unsigned s)
{
    // zero-fill [devValid, bytes): an update without terms in the row batch
    DevSum& d = sum(lane, s).d;
    if (d.devValid >= d.bytes)
        return;
    const unsigned at = sum(lane, s).elementEnd;
    const unsigned lo = std::min(at, windowLo_);
    cover(lo, lo);   // an open batch whose window starts at or below `at`
    prog_.rows_update(lane * kSums + s, d.buf.addr(), d.bytes, d.devValid, s, at, at);
    d.devValid = d.bytes;
}

static uint8_t sum_coeff(unsigned sumIndex, unsigned column)
{
    if (sumIndex == 0)
        return 1;
    const uint8_t cx = column_value(column);
    return sumIndex == 2 ? gf_sqr(cx) : cx;
}

DevSum& DecoderCore::get_sum(unsigned lane, unsigned s, unsigned elementEnd)
{
    Sum& S = sum(lane, s);
    unsigned element = S.elementEnd;
    if (element >= elementEnd)
        return S.d;

    // (the three sums of a lane usually walk the same elements: the walk's
    // result is kept per lane for the next of them)
    LaneScan& ls = laneScan_[lane];
    unsigned end = element;
    if (!(ls.from == element && ls.to == elementEnd && ls.epoch == scanEpoch_)) {
        unsigned most = 0, cnt = 0;
        for (; end < elementEnd; end += kLanes) {
            const unsigned b = slot(end).bytes;
            if (b > 0) {
                most = std::max(most, b);
                ++cnt;
            }
        }
        ls.from = element;
        ls.to = elementEnd;
        ls.end = end;
        ls.most = most;
        ls.got = cnt;
        ls.epoch = scanEpoch_;
    }
    end = ls.end;
    const unsigned got = ls.got;
    const unsigned newBytes = std::max(S.d.bytes, ls.most);
    if (got > 0) {
        if (!grow_sum(S.d, newBytes))
            return S.d;
        // terms (received originals; lost ones are absent in the window),
        // their coefficients and their reference source bytes are generated
        // on the device
        cover(std::min(element, windowLo_), end - kLanes + 1);
        prog_.rows_update(lane * kSums + s, S.d.buf.addr(), S.d.bytes, S.d.devValid, s, element, end);
        S.d.devValid = S.d.bytes;
    }
    S.elementEnd = end;
    return S.d;
}

bool DecoderCore::plug_sum_holes(unsigned elementStart)
{
    for (unsigned column : recoveredColumns_) {
        const unsigned element = column_to_element(column);
        if (element >= count_)
            continue;
        const unsigned lane = column % kLanes;
        const unsigned laneStart = next_lane_element(elementStart, lane);
        for (unsigned s = 0; s < kSums; ++s) {
            Sum& S = sum(lane, s);
            if (element < laneStart || element >= S.elementEnd)
                continue;
            const DecSlot& o = slot(element);
            if (o.bytes == 0)
                return false;
            if (!grow_sum(S.d, o.bytes))
                return false;
            prog_.lc_begin(S.d.buf.addr(), S.d.bytes, S.d.devValid);
            prog_.lc_term(o.buf.addr(), o.bytes, sum_coeff(s, column));
            prog_.lc_end();
            account_elim(o.bytes);
            S.d.devValid = S.d.bytes;
        }
    }
    recoveredColumns_.clear();
    return true;
}

void DecoderCore::reset_sums(unsigned elementStart)
{
    for (unsigned lane = 0; lane < kLanes; ++lane) {
        const unsigned laneStart = next_lane_element(elementStart, lane);
        for (unsigned s = 0; s < kSums; ++s) {
            Sum& S = sum(lane, s);
            S.elementStart = laneStart;
            S.elementEnd = laneStart;
            S.d.bytes = 0;
            S.d.devValid = 0;
        }
    }
    recoveredColumns_.clear();
}

bool DecoderCore::start_sums(unsigned elementStart, unsigned bufferBytes)
{
    for (unsigned lane = 0; lane < kLanes; ++lane) {
        const unsigned laneStart = next_lane_element(elementStart, lane);
        for (unsigned s = 0; s < kSums; ++s) {
            Sum& S = sum(lane, s);
            if (S.d.bytes == 0) {
                S.elementEnd = laneStart;
            } else if (S.elementStart != laneStart) {
                S.elementEnd = laneStart;
                S.d.bytes = 0;
                S.d.devValid = 0;
            }
            S.elementStart = laneStart;
            if (!grow_sum(S.d, bufferBytes))
                return false;
        }
    }
    if (!recoveredColumns_.empty() && !plug_sum_holes(elementStart))
        return false;
    return true;
}

// ---------------------------------------------------------------------------
// Window removal (:1778-2033)

void DecoderCore::remove_elements()
{
    if (nextExpected_ < kRemoveThreshold)
        return;

    unsigned firstKept = 0;
    unsigned targetStart = 0, targetCount = 0, initialBytes = 0;
    bool seenSum = false;

    const RecPacket* r = head_;
    if (!r) {
        const RowMeta m = lastMeta_;
        const unsigned end = column_to_element(m.columnStart + m.sumCount);
        if (column_delta_negative(end) || end < m.ldpcCount) {
            disabled_ = true;
            return;
        }
        firstKept = end - m.ldpcCount;
        targetStart = m.columnStart;
        targetCount = m.sumCount;
        initialBytes = lastBytes_;
        if (m.sumCount > kCauchyThreshold)
            seenSum = true;
    } else {
        firstKept = r->elementStart;
        initialBytes = r->bytes;
        for (;;) {
            const unsigned sc = r->meta.sumCount;
            const unsigned cs = r->meta.columnStart;
            if (sc > kCauchyThreshold) {
                if (!seenSum) {
                    targetStart = cs;
                    targetCount = sc;
                    seenSum = true;
                } else if (cs != targetStart || sc < targetCount) {
                    const unsigned firstSum = column_to_element(cs);
                    if (firstSum >= count_) {
                        disabled_ = true;
                        return;
                    }
                    if (firstKept > firstSum)
                        firstKept = firstSum;
                }
            }
            r = r->next;
            if (!r)
                break;
            if (firstKept > r->elementStart)
                firstKept = r->elementStart;
            if (initialBytes < r->bytes)
                initialBytes = r->bytes;
        }
    }

    if (firstKept < kRemoveThreshold)
        return;

    const unsigned keptSub = firstKept / kSubwindow;
    const unsigned removed = keptSub * kSubwindow;

    if (seenSum) {
        unsigned sumElementStart = column_to_element(targetStart);
        if (sumColumnStart_ != targetStart || sumColumnCount_ > targetCount) {
            if (sumElementStart >= count_) {
                disabled_ = true;
                return;
            }
            reset_sums(sumElementStart);
            sumColumnStart_ = targetStart;
            sumColumnCount_ = targetCount;
        } else {
            if (sumElementStart >= count_)
                sumElementStart = 0;
            if (!start_sums(sumElementStart, initialBytes)) {
                disabled_ = true;
                return;
            }
        }
        ++scanEpoch_;
        for (unsigned lane = 0; lane < kLanes; ++lane) {
            for (unsigned s = 0; s < kSums; ++s) {
                get_sum(lane, s, removed);
                Sum& S = sum(lane, s);
                if (S.elementStart >= removed)
                    S.elementStart -= removed;
                else
                    S.elementStart = lane;
                S.elementEnd -= removed;
            }
        }
    } else {
        // Only Cauchy rows remain: stop maintaining running sums
        sumColumnCount_ = 0;
    }

    // window indices shift below: close the open row batch first
    prog_.rows_seal();
    for (unsigned i = 0; i < keptSub; ++i) {
        // (slab slots go with the slab, back to the arena after the flushes
        // that read them; owned buffers stay until their slot is reused)
        DecSubwindow* sw = subwindows_[i].get();
        for (DecSlot& d : sw->slot)
            if (d.inSlab) {
                d.buf = DevBuf();
                d.inSlab = false;
            }
        eng_->slab_release(sw->slab);
        sw->reset();
    }
    std::rotate(subwindows_.begin(), subwindows_.begin() + keptSub, subwindows_.end());

    count_ -= removed;
    columnStart_ = element_to_column(removed);
    nextExpected_ -= removed;

    for (RecPacket* p = head_; p; p = p->next) {
        p->elementEnd -= removed;
        p->elementStart -= removed;
    }
    if (region_.elementStart < removed || region_.nextCheckStart < removed)
        region_reset();
    else {
        region_.elementStart -= removed;
        region_.nextCheckStart -= removed;
    }
    prevNextCheckStart_ = prevNextCheckStart_ > removed ? prevNextCheckStart_ - removed : 0;
}

// ---------------------------------------------------------------------------
// Recovery packet list (:2567-2666)

void DecSubwindowRecycle::operator()(DecSubwindow* w) const
{
    if (!w->clean) {
        w->got = 0;
        w->gotCount = 0;
        w->slab = Slab();
        for (DecSlot& s : w->slot) {
            s.buf = DevBuf();
            s.inSlab = false;
            s.bytes = 0;
            s.column = 0;
            s.header = 0;
            s.pending = false;
            if (s.hostp)
                s.hostp->clear();
        }
        w->clean = true;
    }
    ObjPool<DecSubwindow>::put(w);
}

void DecoderCore::free_packet(RecPacket* r)
{
    eng_->release(r->buf);
    *r = RecPacket();
    ObjPool<RecPacket>::put(r);
}

void DecoderCore::list_insert(RecPacket* r, bool outOfOrder)
{
    RecPacket* prev = tail_;
    RecPacket* next = nullptr;
    const unsigned rs = r->meta.columnStart;
    const unsigned re = r->elementEnd;
    // Keep both edges of the recovery ranges monotone (SiameseDecoder.h:40-50)
    for (; prev; next = prev, prev = prev->prev) {
        const unsigned pe = prev->elementEnd;
        if (re >= pe) {
            if (re > pe)
                break;
            if (column_delta_negative(column_sub(rs, prev->meta.columnStart)))
                break;
        }
    }
    r->next = next;
    r->prev = prev;
    if (prev)
        prev->next = r;
    else
        head_ = r;
    if (next)
        next->prev = r;
    else
        tail_ = r;
    if (!prev || next)
        region_reset(); // a smaller solution may now exist
    ++listCount_;
    if (!outOfOrder) {
        lastMeta_ = r->meta;
        lastBytes_ = r->bytes;
    }
}

void DecoderCore::list_delete_before(unsigned element)
{
    RecPacket* r = head_;
    unsigned deleted = 0;
    bool regionStale = false;
    while (r && r->elementEnd <= element) {
        RecPacket* n = r->next;
        // The reference keeps using a checked region whose packets it has
        // just freed (use-after-free; it crashes under reordered input, see
        // DESIGN.md "Deviations").  Drop such a region instead.
        if (r == region_.first || r == region_.last)
            regionStale = true;
        free_packet(r);
        ++deleted;
        r = n;
    }
    if (regionStale)
        region_reset();
    head_ = r;
    if (r) {
        r->prev = nullptr;
        listCount_ -= deleted;
    } else {
        tail_ = nullptr;
        listCount_ = 0;
    }
}

// ---------------------------------------------------------------------------
// Recovery packets in (:257-539)

SiameseResult DecoderCore::add_recovery(const SiameseRecoveryPacket& packet)
{
    settle();
    if (dead())
        return Siamese_Disabled;
    RowMeta m;
    const int footer = read_footer(packet.Data, packet.DataBytes, &m);
    if (footer < 0) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    return add_recovery_common(m, footer, packet.DataBytes, packet.Data, 0, packet.Data, nullptr);
}

SiameseResult DecoderCore::add_recovery_device(const DeviceRecovery& rec)
{
    settle();
    if (dead())
        return Siamese_Disabled;
    RowMeta m;
    // The footer sits at the end of the packet; the producer handed us a
    // host copy of exactly those bytes.
    int footer = read_footer(rec.footer, rec.footerBytes, &m);
    if (footer < 0 || (unsigned)footer != rec.footerBytes) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    return add_recovery_common(m, footer, rec.bytes, nullptr, rec.data, rec.head, rec.producer);
}

SiameseResult DecoderCore::add_recovery_common(const RowMeta& m, int footer, unsigned totalBytes,
                                               const void* hostData, uint64_t devData,
                                               const uint8_t* headBytes, Program* producer)
{
    stats_[SiameseDecoderStats_RecoveryCount]++;
    stats_[SiameseDecoderStats_RecoveryBytes] += totalBytes;

    const bool outOfOrder = column_delta_negative(m.columnStart + m.sumCount - latestColumn_);
    if (!outOfOrder)
        latestColumn_ = (m.columnStart + m.sumCount) % kColumnPeriod;

    unsigned elementStart, elementEnd;
    if (count_ == 0) {
        if (outOfOrder) {
            stats_[SiameseDecoderStats_DupedRecoveryCount]++;
            return Siamese_Success;
        }
        columnStart_ = m.columnStart;
        grow_window(m.sumCount);
        elementEnd = m.sumCount;
        elementStart = elementEnd - m.ldpcCount;
    } else {
        elementEnd = column_to_element(m.columnStart + m.sumCount);
        if (column_delta_negative(elementEnd) || elementEnd < m.ldpcCount) {
            stats_[SiameseDecoderStats_DupedRecoveryCount]++;
            return Siamese_Success;
        }
        elementStart = elementEnd - m.ldpcCount;
        if (elementEnd <= nextExpected_) {
            if (outOfOrder) {
                stats_[SiameseDecoderStats_DupedRecoveryCount]++;
                return Siamese_Success;
            }
            if (elementStart >= kRemoveThreshold) {
                lastMeta_ = m;
                lastBytes_ = totalBytes - footer;
                remove_elements();
            }
            stats_[SiameseDecoderStats_DupedRecoveryCount]++;
            return Siamese_Success;
        }
        if (m.sumCount > kCauchyThreshold) {
            if (sumColumnCount_ == 0 || sumColumnStart_ != m.columnStart) {
                if (column_to_element(m.columnStart) >= count_) {
                    stats_[SiameseDecoderStats_DupedRecoveryCount]++;
                    return Siamese_Success;
                }
            }
        }
        grow_window(elementEnd);
    }

    const unsigned payload = totalBytes - footer;
    if (m.sumCount == 1) {
        if (!add_single(m, headBytes, payload, hostData, devData, producer)) {
            disabled_ = true;
            return Siamese_Disabled;
        }
        return Siamese_Success;
    }

    RecPacket* r = ObjPool<RecPacket>::get();
    r->buf = eng_->alloc(payload + payload / 16);
    if (!r->buf) {
        ObjPool<RecPacket>::put(r);
        disabled_ = true;
        return Siamese_Disabled;
    }
    static const uint8_t none[1] = {0};
    if (hostData)
        prog_.ingest_host(r->buf, hostData, payload, none, 0);
    else if (!producer)
        // staged from host memory (framed datagrams, sgpu_frames_recv): in
        // place before the submission starts, at any byte alignment
        prog_.ingest_device(r->buf, devData, payload, none, 0);
    else {
        // A device-resident packet may have been encoded in this very flush:
        // copy it with an op of this (group-1) program, which runs after
        // every encoder op of the flush.  Encoders give each packet a fresh
        // buffer, so nothing overwrites it before the copy, and this program
        // never writes it, so the copy can share a batch with others.
        (void)producer;
        prog_.copy(r->buf.addr(), devData, payload);
    }
    r->bytes = payload;
    r->meta = m;
    r->elementStart = elementStart;
    r->elementEnd = elementEnd;
    list_insert(r, outOfOrder);
    if (elementStart >= kRemoveThreshold)
        remove_elements();
    return Siamese_Success;
}

bool DecoderCore::add_single(const RowMeta& m, const uint8_t* headBytes, unsigned payloadBytes,
                             const void* hostData, uint64_t devData, Program* producer)
{
    const unsigned element = column_to_element(m.columnStart);
    if (element >= count_)
        return false;
    DecSlot& s = slot(element);
    if (s.bytes != 0)
        return true; // duplicate of data we already hold

    unsigned length = 0;
    const int headerBytes = read_length_prefix(headBytes, std::min(payloadBytes, kMaxLengthPrefix), &length);
    if (headerBytes < 1 || length == 0 || length + (unsigned)headerBytes != payloadBytes)
        return false;

    uint8_t hdr[kMaxLengthPrefix];
    const unsigned h = write_length_prefix(length, hdr);
    if (!place(element, h + length))
        return false;
    if (hostData)
        prog_.ingest_host(s.buf, (const uint8_t*)hostData + headerBytes, length, hdr, h);
    else if ((unsigned)headerBytes == h && producer) {
        // Same byte alignment: a copy op of this program (see add_recovery_common)
        prog_.copy(s.buf.addr(), devData, h + length);
    } else
        prog_.ingest_device(s.buf, devData + headerBytes, length, hdr, h);
    if (mirror_) {
        s.host().resize(h + length);
        std::memcpy(s.host().data(), hdr, h);
        std::memcpy(s.host().data() + h, (const uint8_t*)hostData + headerBytes, length);
    }
    s.header = h;
    s.bytes = h + length;
    s.column = m.columnStart;
    s.pending = false;

    {
        // (a completion may be patching the previous decode's outputs)
        std::lock_guard<std::mutex> g(res_->mu);
        if (!hasRecovered_) {
            hasRecovered_ = true;
            recovered_.clear();
            ++decodeSerial_;
        }
        SiameseOriginalPacket out;
        out.PacketNum = m.columnStart;
        out.DataBytes = length;
        out.Data = (mirror_ ? s.host().data() : s.buf.ptr) + h;
        recovered_.push_back(out);
        publish_outputs();
    }
    recoveredColumns_.push_back(m.columnStart);

    if (element >= region_.elementStart && element < region_.nextCheckStart)
        region_reset();

    if (mark_got(m.columnStart)) {
        iterate_next_expected(element + 1);
        list_delete_before(nextExpected_);
        if (region_.nextCheckStart >= kRemoveThreshold)
            remove_elements();
    }
    return true;
}

// ---------------------------------------------------------------------------
// Solvability search and decode driver (:541-810)

void DecoderCore::matrix_reset()
{
    cols_.clear();
    rows_.clear();
    pivots_.clear();
    matRows_ = matCols_ = 0;
    prevNextCheckStart_ = 0;
    geResume_ = 0;
}

void DecoderCore::region_reset()
{
    region_.elementStart = 0;
    region_.nextCheckStart = 0;
    region_.first = nullptr;
    region_.last = nullptr;
    region_.recoveryCount = 0;
    region_.lostCount = 0;
    region_.solveFailed = false;
    matrix_reset();
}

bool DecoderCore::check_recovery_possible()
{
    if (dead())
        return false;
    RecPacket* r;
    unsigned nextCheck, recCount, lost;
    if (!region_.last) {
        r = head_;
        if (!r)
            return false;
        region_.first = r;
        region_.elementStart = r->elementStart;
        recCount = 1;
        nextCheck = r->elementEnd;
        lost = range_lost(r->elementStart, nextCheck);
        region_.solveFailed = false;
        r->lostCount = lost;
    } else {
        recCount = region_.recoveryCount;
        lost = region_.lostCount;
        if (recCount >= lost && !region_.solveFailed)
            return lost <= kMaxLossRecovery;
        r = region_.last;
        nextCheck = region_.nextCheckStart;
    }
    while ((recCount < lost || region_.solveFailed) && r->next) {
        r = r->next;
        ++recCount;
        unsigned end = r->elementEnd;
        if (end < nextCheck)
            end = nextCheck;
        lost += range_lost(nextCheck, end);
        nextCheck = end;
        r->lostCount = lost;
        region_.solveFailed = false;
    }
    region_.last = r;
    region_.recoveryCount = recCount;
    region_.lostCount = lost;
    region_.nextCheckStart = nextCheck;
    if (lost > kMaxLossRecovery)
        return false;
    return recCount >= lost && !region_.solveFailed;
}

SiameseResult DecoderCore::is_ready()
{
    settle();
    if (hasRecovered_ || check_recovery_possible())
        return Siamese_Success;
    return Siamese_NeedMoreData;
}

SiameseResult DecoderCore::decode(SiameseOriginalPacket** packetsOut, unsigned* countOut)
{
    settle();
    if (dead())
        return Siamese_Disabled;
    if (hasRecovered_) {
        hasRecovered_ = false;
        if (packetsOut) {
            *packetsOut = recovered_.data();
            *countOut = (unsigned)recovered_.size();
        }
        return Siamese_Success;
    }
    if (packetsOut) {
        *packetsOut = nullptr;
        *countOut = 0;
    }
    if (!check_recovery_possible())
        return Siamese_NeedMoreData;
    return decode_loop(packetsOut, countOut);
}

SiameseResult DecoderCore::decode_loop(SiameseOriginalPacket** packetsOut, unsigned* countOut)
{
    RecPacket* r = region_.last;
    unsigned nextCheck = region_.nextCheckStart;
    unsigned recCount = region_.recoveryCount;
    unsigned lost = region_.lostCount;

    for (;;) {
        if (recCount >= lost) {
            const SiameseResult res = decode_region();
            if (res == Siamese_Success) {
                if (packetsOut) {
                    *packetsOut = recovered_.data();
                    *countOut = (unsigned)recovered_.size();
                }
                return Siamese_Success;
            }
            if (res != Siamese_NeedMoreData)
                return res;
        }
        if (!r->next)
            break;
        r = r->next;
        ++recCount;
        unsigned end = r->elementEnd;
        if (end < nextCheck)
            end = nextCheck;
        lost += range_lost(nextCheck, end);
        r->lostCount = lost;
        nextCheck = end;
    }
    region_.last = r;
    region_.nextCheckStart = nextCheck;
    region_.recoveryCount = recCount;
    region_.lostCount = lost;
    return Siamese_NeedMoreData;
}

namespace {
// SIAMESE_AMD_DECODE_CLOCKS=1: TSC ticks of decode_region's phases, summed
// over all decoders and printed at exit (profiling aid)
const bool kDecodeClocks = std::getenv("SIAMESE_AMD_DECODE_CLOCKS") != nullptr;
struct DecodeClocks
{
    std::atomic<uint64_t> n{0}, rows{0}, cols{0}, fails{0}, fresh{0}, t[4];
    // per-call samples for medians (a noisy host: averages swing with steal time)
    std::mutex mu;
    std::vector<uint32_t> samples[4];
    void sample(const uint64_t* d)
    {
        std::lock_guard<std::mutex> g(mu);
        for (int k = 0; k < 4; ++k)
            if (samples[k].size() < (1u << 16))
                samples[k].push_back((uint32_t)d[k]);
    }
    ~DecodeClocks()
    {
        if (!kDecodeClocks || !n)
            return;
        double med[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k)
            if (!samples[k].empty()) {
                std::nth_element(samples[k].begin(), samples[k].begin() + samples[k].size() / 2, samples[k].end());
                med[k] = samples[k][samples[k].size() / 2];
            }
        std::fprintf(stderr, "decode_region medians (ticks): generate %.0f ge %.0f eliminate %.0f solve %.0f\n",
                     med[0], med[1], med[2], med[3]);
        std::fprintf(stderr, "decode_region %llu solved, %llu failed, %llu fresh matrices, rows %.1f cols %.1f; "
                     "ticks/solved call: generate %.0f ge %.0f eliminate %.0f solve %.0f\n",
                     (unsigned long long)n.load(), (unsigned long long)fails.load(), (unsigned long long)fresh.load(),
                     (double)rows / (n + fails), (double)cols / (n + fails), (double)t[0] / n, (double)t[1] / n,
                     (double)t[2] / n, (double)t[3] / n);
    }
} g_decodeClocks;
// the chained device decode's host phases (same switch): the job's input,
// the elimination of received data, the solve's layout, the finish
struct ChainClocks
{
    std::mutex mu;
    std::vector<uint32_t> samples[4];
    void sample(const uint64_t* d)
    {
        std::lock_guard<std::mutex> g(mu);
        for (int k = 0; k < 4; ++k)
            if (samples[k].size() < (1u << 16))
                samples[k].push_back((uint32_t)d[k]);
    }
    ~ChainClocks()
    {
        if (!kDecodeClocks || samples[0].empty())
            return;
        double med[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k)
            if (!samples[k].empty()) {
                std::nth_element(samples[k].begin(), samples[k].begin() + samples[k].size() / 2, samples[k].end());
                med[k] = samples[k][samples[k].size() / 2];
            }
        std::fprintf(stderr, "chained decode medians (ticks): job %.0f eliminate %.0f solve %.0f finish %.0f\n",
                     med[0], med[1], med[2], med[3]);
    }
} g_chainClocks;
thread_local uint64_t t_chain[3];
} // namespace

SiameseResult DecoderCore::decode_region()
{
    uint64_t c0 = kDecodeClocks ? __rdtsc() : 0, c1 = 0, c2 = 0, c3 = 0;
    const size_t oldRowsAtEntry = rows_.size();
    geBytes_ = 0;   // (generate_matrix may resume an elimination)
    if (!generate_matrix()) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    if (kDecodeClocks)
        c1 = __rdtsc();
    const bool solved = gaussian_elimination();
    eng_->account(geBytes_);
    if (kDecodeClocks) {
        c2 = __rdtsc();
        g_decodeClocks.rows += matRows_;
        g_decodeClocks.cols += matCols_;
        g_decodeClocks.fails += solved ? 0 : 1;
        g_decodeClocks.fresh += oldRowsAtEntry == 0 ? 1 : 0;
    }
    if (!solved)
        return finish_region(false);
    if (!eliminate_original_data()) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    if (kDecodeClocks)
        c3 = __rdtsc();
    const SiameseResult res = solve_and_substitute();
    if (kDecodeClocks) {
        const uint64_t c4 = __rdtsc();
        g_decodeClocks.n++;
        g_decodeClocks.t[0] += c1 - c0;
        g_decodeClocks.t[1] += c2 - c1;
        g_decodeClocks.t[2] += c3 - c2;
        g_decodeClocks.t[3] += c4 - c3;
        const uint64_t d[4] = {c1 - c0, c2 - c1, c3 - c2, c4 - c3};
        g_decodeClocks.sample(d);
    }
    region_reset();
    return res;
}

SiameseResult DecoderCore::finish_region(bool solved)
{
    if (!solved) {
        region_.solveFailed = true;
        stats_[SiameseDecoderStats_SolveFailCount]++;
        return Siamese_NeedMoreData;
    }
    if (!eliminate_original_data()) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    const SiameseResult res = solve_and_substitute();
    region_reset();
    return res;
}

// ---------------------------------------------------------------------------
// The recovery matrix on the device (decode_device, ops.h GeDesc)

SiameseResult DecoderCore::decode_device(SiameseOriginalPacket** packetsOut, unsigned* countOut)
{
    if (geState_)
        return finish_device_ge(packetsOut, countOut);
    settle();
    if (dead())
        return Siamese_Disabled;
    if (hasRecovered_) {
        hasRecovered_ = false;
        if (packetsOut) {
            *packetsOut = recovered_.data();
            *countOut = (unsigned)recovered_.size();
        }
        return Siamese_Success;
    }
    if (packetsOut) {
        *packetsOut = nullptr;
        *countOut = 0;
    }
    if (!check_recovery_possible())
        return Siamese_NeedMoreData;
    // (the search's first attempt, on a fresh matrix: decode_loop's first
    // decode_region)
    if (region_.recoveryCount >= region_.lostCount && rows_.empty() && geResume_ == 0 && !geHost_ &&
        (submit_chained() || submit_device_ge()))
        return kDecodePending;
    return decode_loop(packetsOut, countOut);
}

bool DecoderCore::submit_device_ge(bool chained)
{
    const unsigned columns = region_.lostCount;
    const unsigned rows = region_.recoveryCount;
    if (columns == 0 || columns > kGeMaxCols || rows > kGeMaxRows)
        return false;
    // generate_matrix's bookkeeping on a fresh matrix; the coefficients are
    // the device's
    matrix_resize(rows, columns, true);
    populate_columns(0, columns);
    populate_rows(0, rows);
    unsigned pickLo = ~0u, pickHi = 0;
    for (unsigned i = 0; i < rows; ++i) {
        const RecPacket* rec = rows_[i].rec;
        if (rec->meta.sumCount <= kCauchyThreshold)
            continue;
        pickLo = std::min(pickLo, rec->elementStart);
        pickHi = std::max(pickHi, rec->elementStart + rec->meta.ldpcCount);
    }
    const unsigned pickLen = pickHi > pickLo ? pickHi - pickLo : 0;
    if (disabled_ || pickLen > kGeMaxPick) {
        // (the host path meets the same condition and handles it)
        disabled_ = false;
        matrix_reset();
        return false;
    }
    uint32_t base = 0;
    uint8_t* in = prog_.ge_job(rows, columns, pickLen, &base, chained);
    GeRow* R = reinterpret_cast<GeRow*>(in);
    GeCol* C = reinterpret_cast<GeCol*>(R + rows);
    uint8_t* pick = reinterpret_cast<uint8_t*>(C + columns);
    for (unsigned j = 0; j < columns; ++j)
        C[j] = GeCol{colLane_[j], colCx_[j], colCx2_[j], (uint8_t)(cols_[j].column % kCauchyMaxColumns)};
    for (unsigned e = pickLo; e < pickHi; ++e) {
        const DecSlot& a = slot(e);
        pick[e - pickLo] = (a.bytes == 0 && a.column < columns) ? (uint8_t)a.column : kGeNoColumn;
    }
    // rows of one decode share their column range: the end of the dense
    // part for the last (columnStart, sumCount) is remembered
    unsigned endKeyStart = ~0u, endKeyCount = 0, endVal = 0;
    for (unsigned i = 0; i < rows; ++i) {
        const RecPacket* rec = rows_[i].rec;
        const RowMeta m = rec->meta;
        unsigned jEnd = 0;
        if (endKeyStart == m.columnStart && endKeyCount == m.sumCount)
            jEnd = endVal;
        else {
            while (jEnd < columns && column_sub(cols_[jEnd].column, m.columnStart) < m.sumCount)
                ++jEnd;
            endKeyStart = m.columnStart;
            endKeyCount = m.sumCount;
            endVal = jEnd;
        }
        GeRow& g = R[i];
        std::memset(&g, 0, sizeof(g));
        g.jEnd = (uint16_t)jEnd;
        g.colCount = (uint16_t)rows_[i].columnCount;
        if (m.sumCount <= kCauchyThreshold) {
            g.kind = m.row == 0 ? GE_PARITY : GE_CAUCHY;
            g.rbase = (uint8_t)(m.row - 1 + kCauchyMaxColumns);
        } else {
            g.kind = GE_SIAMESE;
            g.row = (uint16_t)m.row;
            g.ldpcN = m.ldpcCount;
            g.pickOff = rec->elementStart - pickLo;
        }
    }
    const uint32_t words = ge_result_words(rows, columns, chained);
    prog_.on_complete(res_, [r = res_.get(), base, words](const uint32_t* results) {
        std::lock_guard<std::mutex> g(r->mu);
        r->geOut.assign(results + base, results + base + words);
        r->geDone = true;
    });
    geState_ = chained ? 2 : 1;
    EngineStats& st = eng_->shard().stats;
    st.geJobs++;
    st.geChained += chained ? 1 : 0;
    geRows_ = rows;
    geCols_ = columns;
    geBase_ = base;
    return true;
}

// A block decode on the device in one submission.  The first attempt on a
// square matrix (as many recovery rows as lost columns) of Siamese rows of one
// length: whatever pivot order the elimination takes, it uses every row, and
// rows of one length never grow in MultiplyLowerTriangle, so the elimination
// of received data (EliminateOriginalData, SiameseDecoder.cpp:812-1063) and
// the solve's layout do not depend on the coefficients.  Both are queued now,
// gated on the job's outcome word (every op the elimination of received data
// emits -- row batches with their sum updates, Cauchy rows, sum growth -- and
// the solve run only if the device elimination succeeds; otherwise the
// host's sums go back to their state before it, chain_sums_restore), and the
// job writes the solve's coefficients and row order itself.  The host side of
// BackSubstitution waits for finish_chained.  Siamese rows of wide LDPC sums
// are not chained (their k_ldpc items are not gated).
bool DecoderCore::submit_chained()
{
    const unsigned columns = region_.lostCount;
    const unsigned rows = region_.recoveryCount;
    if (mirror_ || rows != columns || columns == 0 || columns > kGeMaxCols)
        return false;
    const uint64_t c0 = kDecodeClocks ? __rdtsc() : 0;
    const RecPacket* r = region_.first;
    const unsigned bytes = r->bytes;
    for (unsigned i = 0; i < rows; ++i, r = r->next)
        if ((r->meta.sumCount > kCauchyThreshold && r->meta.ldpcCount >= kLdpcSplitMin) || r->bytes != bytes)
            return false;
    if (!submit_device_ge(true))
        return false;
    const uint64_t c1 = kDecodeClocks ? __rdtsc() : 0;
    pivots_.resize(rows);
    for (unsigned i = 0; i < rows; ++i) {
        rows_[i].used = true;
        pivots_[i] = i;
    }
    const uint32_t okWord = geBase_ + 3;   // (ops.h GeDesc: 1 once eliminated)
    for (unsigned l = 0; l < kLanes; ++l)
        for (unsigned k = 0; k < kSums; ++k)
            chainSums_.lanes[l][k] = lanes_[l][k];
    chainSums_.columnStart = sumColumnStart_;
    chainSums_.columnCount = sumColumnCount_;
    chainSums_.recoveredColumns = recoveredColumns_;
    chainReleases_.clear();
    prog_.gate_begin(okWord);
    deferAccount_ = true;
    deferRelease_ = true;
    deferredBytes_ = 0;
    chainElimFailed_ = !eliminate_original_data();
    deferAccount_ = false;
    deferRelease_ = false;
    prog_.gate_end();
    const uint64_t c2 = kDecodeClocks ? __rdtsc() : 0;
    chainSlot_ = ~0u;
    chainBytes_ = bytes;
    if (!chainElimFailed_) {
        unsigned slot = 0;
        if (solve_plan(okWord + 1, &slot))
            chainSlot_ = slot;
        else
            chainElimFailed_ = true;   // (an arena failure: disabled_ is set)
    }
    if (kDecodeClocks) {
        t_chain[0] = c1 - c0;
        t_chain[1] = c2 - c1;
        t_chain[2] = __rdtsc() - c2;
    }
    return true;
}

SiameseResult DecoderCore::finish_chained(SiameseOriginalPacket** packetsOut, unsigned* countOut)
{
    const unsigned columns = geCols_;
    const uint32_t* o = geOut_.data();
    const bool ok = o[3] != 0;
#ifdef SGPU_GE_CLOCKS
    // (timing build: k_ge's phases in 100 MHz ticks, averaged at exit)
    static struct GeClocks
    {
        std::atomic<uint64_t> n{0}, t[3];
        std::mutex mu;
        std::vector<std::pair<uint32_t, uint32_t>> jobs;   // (ticks, columns)
        ~GeClocks()
        {
            if (!n)
                return;
            std::fprintf(stderr, "k_ge phases (us): staging %.2f generate %.2f eliminate %.2f over %llu jobs\n",
                         t[0] / 100.0 / n, t[1] / 100.0 / n, t[2] / 100.0 / n, (unsigned long long)n.load());
            std::sort(jobs.begin(), jobs.end());
            for (double q : {0.5, 0.9, 0.99, 1.0}) {
                const auto& j = jobs[std::min(jobs.size() - 1, (size_t)(q * jobs.size()))];
                std::fprintf(stderr, "k_ge job q%.2f: %.2f us, %u columns\n", q, j.first / 100.0, j.second);
            }
        }
    } clocks;
    clocks.n++;
    for (int k = 0; k < 3; ++k)
        clocks.t[k] += o[5 + k];
    {
        std::lock_guard<std::mutex> g(clocks.mu);
        clocks.jobs.emplace_back(o[5] + o[6] + o[7], columns);
    }
#endif
    const uint64_t f0 = kDecodeClocks ? __rdtsc() : 0;
    auto drop_solve = [&] {
        // the planned solve did not run (or is not wanted): its slot goes
        // back without touching the decoder's state
        if (chainSlot_ == ~0u)
            return;
        std::lock_guard<std::mutex> g(res_->mu);
        PendingDecode& pd = res_->pend[chainSlot_];
        if (pd.done)
            ++appliedCount_;   // (its completion counted in doneCount)
        pd.live = pd.done = pd.held = false;
        pendingSolves_--;
        chainSlot_ = ~0u;
    };
    if (dead()) {
        drop_solve();
        chain_sums_commit();
        return Siamese_Disabled;
    }
    if (!ok) {
        // a singular matrix: nothing gated ran (the elimination of received
        // data, its sum updates, the solve).  The sums go back to their state
        // before it, the host repeats the elimination (the resumable state
        // the reference keeps for the next attempt) and the search goes on
        // as decode() does.
        drop_solve();
        chain_sums_restore();
        eng_->shard().stats.geRetried++;
        geHost_ = true;
        matrix_reset();
        return decode_loop(packetsOut, countOut);
    }
    chain_sums_commit();
    // the device's muladds: the elimination's, the rows' (deferred), the
    // lower triangle's (MultiplyLowerTriangle: rows of one length, non-zero
    // multipliers x that length)
    eng_->account(((uint64_t)o[2] << 32) | o[1]);
    eng_->account(deferredBytes_);
    eng_->account((uint64_t)o[4] * chainBytes_, 0, true);
    if (chainElimFailed_) {
        drop_solve();
        disabled_ = true;
        return Siamese_Disabled;
    }
    const uint8_t* piv = reinterpret_cast<const uint8_t*>(o + ge_out_pivots(geRows_));
    scratchRec_.resize(columns);
    scratchLen_.resize(columns);
    for (unsigned i = 0; i < columns; ++i) {
        pivots_[i] = piv[i];
        scratchRec_[i] = rows_[piv[i]].rec;
        scratchLen_[i] = chainBytes_;
    }
    const unsigned slot = chainSlot_;
    chainSlot_ = ~0u;
    const SiameseResult res = publish_final(slot);
    region_reset();
    if (kDecodeClocks) {
        const uint64_t d[4] = {t_chain[0], t_chain[1], t_chain[2], __rdtsc() - f0};
        g_chainClocks.sample(d);
    }
    if (res == Siamese_Success && packetsOut) {
        *packetsOut = recovered_.data();
        *countOut = (unsigned)recovered_.size();
    }
    return res;
}

SiameseResult DecoderCore::finish_device_ge(SiameseOriginalPacket** packetsOut, unsigned* countOut)
{
    {
        std::lock_guard<std::mutex> g(res_->mu);
        if (!res_->geDone) {
            // A failed submission delivers no completions (Engine::wait), so
            // the job's result never arrives: give the decoder back as the
            // reference's EmergencyDisabled would, instead of pending forever.
            if (!dead())
                return kDecodePending;   // (its flush has not completed yet)
            if (geState_ == 2 && chainSlot_ != ~0u) {
                PendingDecode& pd = res_->pend[chainSlot_];
                pd.live = pd.done = pd.held = false;
                pendingSolves_--;
                chainSlot_ = ~0u;
            }
            geState_ = 0;
            if (packetsOut) {
                *packetsOut = nullptr;
                *countOut = 0;
            }
            return Siamese_Disabled;
        }
        geOut_.swap(res_->geOut);
        res_->geDone = false;
    }
    const bool chained = geState_ == 2;
    geState_ = 0;
    settle();
    if (packetsOut) {
        *packetsOut = nullptr;
        *countOut = 0;
    }
    if (chained)
        return finish_chained(packetsOut, countOut);
    if (dead())
        return Siamese_Disabled;
    const unsigned rows = geRows_, columns = geCols_;
    const uint32_t* o = geOut_.data();
    if (o[0] < columns) {
        // the elimination stopped short of a pivot: the host repeats it (the
        // resumable state the reference keeps for the next attempt), and the
        // search goes on as decode() does
        geHost_ = true;
        matrix_reset();
        return decode_loop(packetsOut, countOut);
    }
    const uint8_t* piv = reinterpret_cast<const uint8_t*>(o + ge_out_pivots(rows));
    const uint8_t* used = reinterpret_cast<const uint8_t*>(o + ge_out_used(rows));
    const uint16_t* cnt = reinterpret_cast<const uint16_t*>(o + ge_out_counts(rows));
    const uint8_t* mat = reinterpret_cast<const uint8_t*>(o + ge_out_matrix(rows));
    pivots_.resize(rows);
    for (unsigned i = 0; i < rows; ++i) {
        pivots_[i] = piv[i];
        rows_[i].used = used[i] != 0;
        rows_[i].columnCount = cnt[i];
        std::memcpy(mrow(i), mat + (size_t)i * columns, columns);
    }
    geBytes_ = ((uint64_t)o[2] << 32) | o[1];
    eng_->account(geBytes_);
    const SiameseResult res = finish_region(true);
    if (res == Siamese_Success && packetsOut) {
        *packetsOut = recovered_.data();
        *countOut = (unsigned)recovered_.size();
    }
    return res;
}

void DecoderCore::chain_sums_commit()
{
    for (DevBuf& b : chainReleases_)
        eng_->release(b);
    chainReleases_.clear();
}

void DecoderCore::chain_sums_restore()
{
    // buffers the elimination allocated (grown sums) go back; the ones it
    // replaced are the snapshot's again
    auto in_snapshot = [&](const uint8_t* p) {
        for (unsigned l = 0; l < kLanes; ++l)
            for (unsigned k = 0; k < kSums; ++k)
                if (chainSums_.lanes[l][k].d.buf.ptr == p)
                    return true;
        return false;
    };
    for (DevBuf& b : chainReleases_)
        if (b && !in_snapshot(b.ptr))
            eng_->release(b);
    chainReleases_.clear();
    for (unsigned l = 0; l < kLanes; ++l)
        for (unsigned k = 0; k < kSums; ++k) {
            Sum& S = lanes_[l][k];
            if (S.d.buf && !in_snapshot(S.d.buf.ptr))
                eng_->release(S.d.buf);
            S = chainSums_.lanes[l][k];
        }
    sumColumnStart_ = chainSums_.columnStart;
    sumColumnCount_ = chainSums_.columnCount;
    recoveredColumns_ = chainSums_.recoveredColumns;
    ++scanEpoch_;   // (get_sum's lane walks were of the discarded state)
}

// ---------------------------------------------------------------------------
// Recovery matrix on coefficients (:2039-2531)

bool DecoderCore::matrix_resize(unsigned rows, unsigned columns, bool initialize)
{
    // GrowingAlignedByteMatrix semantics (reference SiameseCommon.cpp:51-117).
    // 64 bytes more than the reference's stride: the elimination's 64-byte
    // masked row stores then never cover the next row's pivot byte, which a
    // store-to-load forward cannot serve (a 3-4x stall per row update), and
    // generate_matrix has spare bytes past the columns
    const unsigned stride = align_up(columns + 4) + 64;
    if (initialize) {
        matAllocRows_ = rows + 4;
        matStride_ = stride;
        mat_.resize((size_t)matAllocRows_ * matStride_ + kRowSlack);
    } else if (!(rows <= matAllocRows_ && columns + 4 <= matStride_)) {   // (a spare byte per row, generate_matrix)
        std::vector<uint8_t> nm((size_t)(rows + 4) * stride + kRowSlack);
        const unsigned copy = std::min(matCols_, columns);
        if (matCols_ > 0)
            for (unsigned i = 0; i < matRows_; ++i)
                std::memcpy(nm.data() + (size_t)i * stride, mat_.data() + (size_t)i * matStride_, copy);
        mat_.swap(nm);
        matAllocRows_ = rows + 4;
        matStride_ = stride;
    }
    matRows_ = rows;
    matCols_ = columns;
    return true;
}

void DecoderCore::populate_columns(unsigned oldColumns, unsigned newColumns)
{
    if (oldColumns >= newColumns)
        return;
    cols_.resize(newColumns);
    colLane_.resize(newColumns + kRowSlack);
    colCx_.resize(newColumns + kRowSlack);
    colCx2_.resize(newColumns + kRowSlack);
    unsigned elementStart = prevNextCheckStart_;
    prevNextCheckStart_ = region_.nextCheckStart;
    const unsigned elementEnd = region_.nextCheckStart;
    if (elementStart < region_.elementStart)
        elementStart = region_.elementStart;
    const unsigned subEnd = (elementEnd + kSubwindow - 1) / kSubwindow;
    unsigned sub = elementStart / kSubwindow;
    unsigned bit = elementStart % kSubwindow;
    unsigned column = oldColumns;
    while (sub < subEnd) {
        DecSubwindow* sw = subwindows_[sub].get();
        if (sw->gotCount < kSubwindow) {
            do {
                bit = first_clear(sw->got, bit);
                if (bit >= kSubwindow)
                    break;
                ColInfo& c = cols_[column];
                c.column = element_to_column(sub * kSubwindow + bit);
                c.original = &sw->slot[bit];
                const uint8_t cx = column_value(c.column);
                colLane_[column] = (uint8_t)(c.column % kLanes);
                colCx_[column] = cx;
                colCx2_[column] = gf_sqr(cx);
                c.original->column = column; // lost slot -> matrix column
                if (++column >= newColumns)
                    return;
            } while (++bit < kSubwindow);
        }
        bit = 0;
        ++sub;
    }
    disabled_ = true; // ran out of lost columns: should never happen
}

void DecoderCore::populate_rows(unsigned oldRows, unsigned newRows)
{
    if (oldRows >= newRows)
        return;
    rows_.resize(newRows);
    RecPacket* r = oldRows > 0 ? rows_[oldRows - 1].rec->next : region_.first;
    for (unsigned i = oldRows; i < newRows; ++i, r = r->next) {
        rows_[i].rec = r;
        rows_[i].used = false;
        rows_[i].columnCount = r->lostCount;
    }
}

bool DecoderCore::generate_matrix()
{
    const unsigned columns = region_.lostCount;
    const unsigned rows = region_.recoveryCount;
    unsigned oldRows = (unsigned)rows_.size();
    unsigned oldColumns = (unsigned)cols_.size();
    if (rows < oldRows || columns < oldColumns) {
        matrix_reset();
        oldRows = 0;
        oldColumns = 0;
    }
    matrix_resize(rows, columns, oldRows == 0);
    populate_columns(oldColumns, columns);
    populate_rows(oldRows, rows);

    const unsigned startRow = (columns <= oldColumns) ? oldRows : 0;

    // The sparse picks only land on lost slots: one pass over the elements
    // the new rows span gives each its matrix column (kNoColumn: received),
    // so the picks below read a small dense array instead of window slots.
    constexpr uint32_t kNoColumn = ~0u;
    unsigned pickLo = ~0u, pickHi = 0;
    for (unsigned i = startRow; i < rows; ++i) {
        const RecPacket* rec = rows_[i].rec;
        if (rec->meta.sumCount <= kCauchyThreshold)
            continue;
        pickLo = std::min(pickLo, rec->elementStart);
        pickHi = std::max(pickHi, rec->elementStart + rec->meta.ldpcCount);
    }
    if (pickHi > pickLo) {
        pickCol_.resize(pickHi - pickLo);
        for (unsigned e = pickLo; e < pickHi; ++e) {
            const DecSlot& a = slot(e);
            pickCol_[e - pickLo] = a.bytes == 0 ? a.column : kNoColumn;
        }
    }
    // rows of one decode share their column range: the end of the dense
    // part for the last (columnStart, sumCount, startCol) is remembered
    unsigned endKeyStart = ~0u, endKeyCount = 0, endKeyFrom = 0, endVal = 0;
    for (unsigned i = startRow; i < rows; ++i) {
        uint8_t* row = mrow(i);
        const RecPacket* rec = rows_[i].rec;
        const RowMeta m = rec->meta;
        const unsigned startCol = (i < oldRows) ? oldColumns : 0;

        if (m.sumCount <= kCauchyThreshold) {
            for (unsigned j = startCol; j < columns; ++j) {
                const unsigned column = cols_[j].column;
                if (column_sub(column, m.columnStart) >= m.sumCount) {
                    std::memset(row + j, 0, columns - j);
                    break;
                }
                row[j] = m.row == 0 ? 1 : cauchy_element(m.row - 1, column % kCauchyMaxColumns);
            }
            continue;
        }

        // Dense coefficient of column x in row r: the opcode's low three bits
        // select {1, CX, CX^2} for the row sum, the high three the same for
        // the product, which is scaled by RX:  v = comb[op&7] ^ RX*comb[op>>3]
        const uint8_t rx = row_value(m.row);
        const RowSelect& sel = row_select(m.row);
        const uint8_t* opLo = sel.opLo;
        const uint8_t* opHi = sel.opHi;
        unsigned jEnd = startCol;
        if (endKeyStart == m.columnStart && endKeyCount == m.sumCount && endKeyFrom == startCol)
            jEnd = endVal;
        else {
            while (jEnd < columns && column_sub(cols_[jEnd].column, m.columnStart) < m.sumCount)
                ++jEnd;
            endKeyStart = m.columnStart;
            endKeyCount = m.sumCount;
            endKeyFrom = startCol;
            endVal = jEnd;
        }
        if (jEnd > startCol)
            gf_dense_row(row + startCol, colLane_.data() + startCol, colCx_.data() + startCol,
                         colCx2_.data() + startCol, opLo, opHi, rx, jEnd - startCol);
        if (jEnd < columns)
            std::memset(row + jEnd, 0, columns - jEnd);

        // Sparse columns that landed on lost data.  A pick on a received
        // original (or on a column this row already has) adds nothing.
        const uint32_t* pc = pickCol_.data() + (rec->elementStart - pickLo);
        const uint32_t span = columns - startCol;
        uint64_t hit1 = 0, hitRx = 0;
        unsigned picks = 0;
        const uint32_t* off = nullptr;
        if (columns <= 64 && (off = ldpc_offsets(m.row, m.ldpcCount, &picks)) != nullptr) {
            // XOR-ing 1 (even picks) or RX (odd picks) into a byte any number
            // of times is the parity of its hits: a bit per column each, in
            // registers (no byte read-modify-write chains through memory)
            for (unsigned k = 0; k + 1 < picks; k += 2) {
                const uint32_t c0 = pc[off[k]], c1 = pc[off[k + 1]];
                hit1 ^= (uint64_t)(c0 - startCol < span) << (c0 & 63);
                hitRx ^= (uint64_t)(c1 - startCol < span) << (c1 & 63);
            }
            for (uint64_t b = hit1 | hitRx; b; b &= b - 1) {
                const unsigned j = (unsigned)__builtin_ctzll(b);
                row[j] ^= (uint8_t)(((hit1 >> j) & 1) ^ (((hitRx >> j) & 1) ? rx : 0));
            }
        } else {
            // (eight spare bytes past `columns` take the picks that land
            // nowhere, so they do not chain through one byte's
            // load-xor-store; they are outside the matrix, rewritten if it
            // ever grows over them)
            off = ldpc_offsets(m.row, m.ldpcCount, &picks);
            const uint8_t val[2] = {1, rx};
            for (unsigned k = 0; k < picks; ++k) {
                const uint32_t c = pc[off[k]];
                const uint32_t at = (c - startCol < span) ? c : columns + (k & 7);
                row[at] ^= val[k & 1];
            }
        }
    }

    pivots_.resize(rows);
    for (unsigned i = oldRows; i < rows; ++i)
        pivots_[i] = i;
    if (geResume_ > 0)
        resume_ge(oldRows, rows);
    return true;
}

namespace {
const bool kGfni = (gf_init(), gf_gfni());
} // namespace

bool DecoderCore::eliminate_row(const uint8_t* geRow, uint8_t* remRow, unsigned pivot, unsigned end,
                                uint8_t valI)
{
    // SiameseDecoder.h:522-541
    const uint8_t valJ = remRow[pivot];
    if (valJ == 0)
        return false;
    const uint8_t y = gf_div(valJ, valI);
    remRow[pivot] = y;
    if (end > pivot + 1) {
        if (kGfni) {   // one affine multiply per 64 bytes (gf.h)
            gf_muladd_fast(remRow + pivot + 1, geRow + pivot + 1, y, end - pivot - 1);
            geBytes_ += end - pivot - 1;
            return true;
        }
        // the pivot row's bytes after the pivot, split into nibbles once for
        // every row it eliminates (geSrcFor_ names the split in geSrc_)
        if (geSrcRow_ != geRow || geSrcPivot_ != pivot || geSrc_.n != end - pivot - 1) {
            gf_row_prepare(geSrc_, geRow + pivot + 1, end - pivot - 1);
            geSrcRow_ = geRow;
            geSrcPivot_ = pivot;
        }
        gf_muladd_prepared(remRow + pivot + 1, geSrc_, y);
        geBytes_ += end - pivot - 1;   // the reference's MulAddRows muladd (:504-520)
    }
    return true;
}

void DecoderCore::resume_ge(unsigned oldRows, unsigned rows)
{
    if (oldRows >= rows)
        return;
    geSrcRow_ = nullptr;
    for (unsigned p = 0; p < geResume_; ++p) {
        const unsigned ri = pivots_[p];
        const uint8_t* ge = mrow(ri);
        const uint8_t val = ge[p];
        const unsigned end = rows_[ri].columnCount;
        for (unsigned k = oldRows; k < rows; ++k)
            if (eliminate_row(ge, mrow(k), p, end, val) && rows_[k].columnCount < end)
                rows_[k].columnCount = end;
    }
}

bool DecoderCore::gaussian_elimination()
{
    geSrcRow_ = nullptr;   // (the matrix may have moved since the last elimination)
    if (geResume_ > 0)
        return pivoted_ge(geResume_);
    const unsigned columns = matCols_;
    const unsigned rows = matRows_;
    {
        // the whole loop in one vector routine where the host has GFNI
        geEnd_.resize(columns);
        for (unsigned p = 0; p < columns; ++p)
            geEnd_[p] = rows_[p].columnCount;
        bool done = false;
        const unsigned stop = gf_ge_nopivot(mat_.data(), matStride_, rows, columns, 0, geEnd_.data(), &geBytes_, &done);
        if (done) {
            for (unsigned p = 0; p < stop; ++p)
                rows_[p].used = true;
            return stop < columns ? pivoted_ge(stop) : true;
        }
    }
    for (unsigned p = 0; p < columns; ++p) {
        uint8_t* ge = mrow(p);
        const uint8_t val = ge[p];
        if (val == 0)
            return pivoted_ge(p);
        rows_[p].used = true;
        const unsigned end = rows_[p].columnCount;
        for (unsigned k = p + 1; k < rows; ++k)
            eliminate_row(ge, mrow(k), p, end, val);
    }
    return true;
}

bool DecoderCore::pivoted_ge(unsigned pivot)
{
    const unsigned columns = matCols_;
    const unsigned rows = matRows_;
    unsigned j = pivot + 1; // the caller already found column `pivot` zero here
    bool resume = true;
    for (; pivot < columns; ++pivot) {
        if (!resume)
            j = pivot;
        resume = false;
        bool found = false;
        for (; j < rows; ++j) {
            const unsigned rj = pivots_[j];
            const uint8_t* ge = mrow(rj);
            const uint8_t val = ge[pivot];
            if (val == 0)
                continue;
            if (pivot != j)
                std::swap(pivots_[pivot], pivots_[j]);
            rows_[rj].used = true;
            const unsigned end = rows_[rj].columnCount;
            if (pivot >= columns - 1)
                return true;
            for (unsigned k = pivot + 1; k < rows; ++k) {
                const unsigned rk = pivots_[k];
                if (eliminate_row(ge, mrow(rk), pivot, end, val) && rows_[rk].columnCount < end)
                    rows_[rk].columnCount = end;
            }
            found = true;
            break;
        }
        if (!found) {
            geResume_ = pivot;
            return false;
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// Eliminate received data from the used rows (:812-1063)

bool DecoderCore::eliminate_original_data()
{
    ++scanEpoch_;   // (get_sum's lane walks are reused within this call only)
    const unsigned rows = region_.recoveryCount;
    // the current run of rows with one sum range (see below)
    bool haveRun = false;
    unsigned runStart = 0, runCount = 0, runEnd = 0, runBytes = 0, runSumStart = 0;
    uint32_t fresh = 0;   // sums brought up to runEnd during this run
    // the 24 sums as rows read them, rebuilt only after a sum may have changed
    WinEntry sums[kRowSums];
    uint32_t clip[kRowSums];   // min(sum bytes, row bytes): reference source bytes
    uint32_t present = 0;      // sums holding bytes
    bool tableStale = true;
    uint64_t tableVersion = 0;   // Program::rows_row's tag of `sums` as last rebuilt
    for (unsigned ri = 0; ri < rows; ++ri) {
        if (!rows_[ri].used)
            continue;
        RecPacket* rec = rows_[ri].rec;
        const RowMeta m = rec->meta;
        const unsigned es = rec->elementStart;
        const unsigned ee = rec->elementEnd;
        const unsigned rb = rec->bytes;

        if (m.sumCount <= kCauchyThreshold) {
            prog_.lc_begin(rec->buf.addr(), rb, rb);
            for (unsigned j = es; j < ee; ++j) {
                const DecSlot& o = slot(j);
                if (o.bytes == 0)
                    continue;
                const uint8_t y = m.row == 0 ? 1 : cauchy_element(m.row - 1, o.column % kCauchyMaxColumns);
                prog_.lc_term(o.buf.addr(), std::min(o.bytes, rb), y);
                account_elim(std::min(o.bytes, rb));
            }
            prog_.lc_end();
            continue;
        }

        // Rows of one decode usually share their sum range (a block of
        // Siamese rows: same ColumnStart/SumCount/end/length).  The restart
        // below is then a no-op for every row after the first, and only sums
        // no earlier row of the run brought up to `ee` need the lazy walk.
        const bool sameRun = haveRun && m.columnStart == runStart && m.sumCount == runCount &&
                             ee == runEnd && rb == runBytes && recoveredColumns_.empty();
        unsigned sumElementStart = column_to_element(m.columnStart);
        if (!sameRun) {
            if (m.columnStart != sumColumnStart_ || m.sumCount < sumColumnCount_) {
                if (sumElementStart >= count_)
                    return false;
                reset_sums(sumElementStart);
                sumColumnStart_ = m.columnStart;
            } else {
                if (sumElementStart >= count_)
                    sumElementStart = 0;
                if (!start_sums(sumElementStart, rb))
                    return false;
            }
            sumColumnCount_ = m.sumCount;
            haveRun = true;
            runStart = m.columnStart;
            runCount = m.sumCount;
            runEnd = ee;
            runBytes = rb;
            fresh = 0;
            tableStale = true;
            runSumStart = sumElementStart;
        }

        // decoder sums first (their updates precede the batch's rows); the
        // row selects them by mask bit lane*3 + sum
        windowLo_ = std::min(es, runSumStart);
        const RowSelect& sel = row_select(m.row);
        const uint32_t want = sel.mask[0] | sel.mask[1];
        uint32_t need = want & ~fresh;
        if (need)
            tableStale = true;   // a sum may grow below: rebuild the table
        for (; need; need &= need - 1) {
            const unsigned k = (unsigned)__builtin_ctz(need);
            if (get_sum(k / kSums, k % kSums, ee).bytes > 0)
                materialize(k / kSums, k % kSums);
        }
        fresh |= want;
        if (tableStale) {
            tableStale = false;
            tableVersion = Program::next_table_version();
            present = 0;
            for (unsigned k = 0; k < kRowSums; ++k) {
                const DevSum& d = sum(k / kSums, k % kSums).d;
                WinEntry& t = sums[k];
                t.src = d.buf.addr();
                t.len = d.bytes;
                t.column = 0;
                if (d.bytes > 0)
                    present |= 1u << k;
                clip[k] = std::min(d.bytes, rb);
            }
        }
        uint64_t opBytes = rb;  // RX * product muladd
        for (uint32_t b = sel.mask[0] & present; b; b &= b - 1)
            opBytes += clip[__builtin_ctz(b)];
        for (uint32_t b = sel.mask[1] & present; b; b &= b - 1)
            opBytes += clip[__builtin_ctz(b)];
        const uint32_t mask[2] = {sel.mask[0] & present, sel.mask[1] & present};
        // LDPC pairs over received originals: drawn (and their reference
        // source bytes counted) on the device
        // rows of one decode share the sums: one row of the program's batch
        cover(windowLo_, ee);
        prog_.rows_row(sums, rec->buf.addr(), rb, rb, row_value(m.row), mask[0], mask[1], m.row,
                       m.ldpcCount, es, ee, nullptr, 0, tableVersion);
        account_elim(opBytes);
    }
    // the window snapshot must not see this decode's recoveries
    prog_.rows_seal();
    return !disabled_;
}

// ---------------------------------------------------------------------------
// Lower-triangle multiply + back-substitution (:1065-1238) as one device solve

SiameseResult DecoderCore::solve_and_substitute()
{
    unsigned slot = 0;
    if (!solve_plan(0, &slot)) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    return solve_publish(slot);
}

bool DecoderCore::solve_plan(uint32_t gateWord, unsigned* slotOut)
{
    const unsigned m = region_.lostCount;
    // (scratch vectors are members: a decode allocates nothing once warm)
    std::vector<RecPacket*>& pr = scratchRec_;
    std::vector<unsigned>& len = scratchLen_;
    pr.resize(m);
    len.resize(m);
    for (unsigned i = 0; i < m; ++i) {
        pr[i] = rows_[pivots_[i]].rec;
        len[i] = pr[i]->bytes;
    }
    // the queued solve's own descriptors and coefficients, filled in place
    SolveRow* desc = nullptr;
    uint8_t* coefOut = nullptr;
    prog_.solve_reserve(m, &desc, &coefOut);
    for (unsigned i = 0; i < m; ++i) {
        std::memset(&desc[i], 0, sizeof(SolveRow));
        desc[i].initBytes = len[i];
    }
    // Row growth of MultiplyLowerTriangle (GrowZeroPadded), simulated here
    uint64_t lowerOpBytes = 0;
    bool equal = true;
    for (unsigned i = 1; i < m && equal; ++i)
        equal = len[i] == len[0];
    if (equal) {
        // rows of one length (a block of equal packets) never grow: the
        // lower step's source bytes are that length per non-zero multiplier
        // below the diagonal, counted a row at a time (a chained solve's by
        // its device elimination, finish_chained)
        if (!gateWord) {
            uint64_t nz = 0;
            for (unsigned j = 1; j < m; ++j)
                nz += gf_count_nonzero(mrow(pivots_[j]), j);
            lowerOpBytes = nz * (m ? len[0] : 0);
        }
        for (unsigned i = 0; i + 1 < m; ++i)
            desc[i].lowerLen = len[i];
    } else {
        for (unsigned i = 0; i + 1 < m; ++i) {
            desc[i].lowerLen = len[i];
            for (unsigned j = i + 1; j < m; ++j) {
                if (mrow(pivots_[j])[i] == 0)
                    continue;
                lowerOpBytes += len[i];
                if (len[j] < len[i])
                    len[j] = len[i];
            }
        }
    }
    if (lowerOpBytes)
        eng_->account(lowerOpBytes, 0, true);
    if (m > 0)
        desc[m - 1].lowerLen = len[m - 1];

    uint32_t maxBytes = 0;
    for (unsigned i = 0; i < m; ++i) {
        RecPacket* r = pr[i];
        if (len[i] > r->buf.cap) {
            DevBuf nb = eng_->alloc(len[i]);
            if (!nb)
                return false;
            prog_.lc_begin(nb.addr(), desc[i].initBytes, 0);
            prog_.lc_term(r->buf.addr(), desc[i].initBytes, 1);
            prog_.lc_end();
            eng_->release(r->buf);
            r->buf = nb;
        }
        desc[i].buf = r->buf.addr();
        desc[i].finalBytes = len[i];
        maxBytes = std::max(maxBytes, len[i]);
    }
    // (a chained solve's coefficients come from its device elimination)
    if (!gateWord)
        for (unsigned j = 0; j < m; ++j)
            std::memcpy(coefOut + (size_t)j * m, mrow(pivots_[j]), m);

    const uint32_t base = prog_.solve_commit(maxBytes, gateWord);

    // a slot for this solve's completion state; a chained solve's is held
    // (apply_resolved leaves it alone) until solve_publish
    unsigned slot = 0;
    {
        std::lock_guard<std::mutex> g(res_->mu);
        std::vector<PendingDecode>& pend = res_->pend;
        while (slot < pend.size() && pend[slot].live)
            ++slot;
        if (slot == pend.size())
            pend.emplace_back();
        PendingDecode& pd = pend[slot];
        pd.live = true;
        pd.done = false;
        pd.held = gateWord != 0;
        pd.base = base;
        pd.m = m;
        pd.serial = ~0ull;   // (no output array of its own until published)
        pd.words.clear();
        pd.targets.clear();
        pd.fixes.clear();
    }
    pendingSolves_++;
    // (the back-substitution's reference source bytes need the recovered
    // lengths: the solve kernel counts them, SiameseDecoder.cpp:1131-1212)
    prog_.on_complete(res_, [r = res_.get(), slot](const uint32_t* results) { complete_solve(*r, slot, results); });
    *slotOut = slot;
    return true;
}

SiameseResult DecoderCore::solve_publish(unsigned slot)
{
    const unsigned m = region_.lostCount;
    const std::vector<RecPacket*>& pr = scratchRec_;
    const std::vector<unsigned>& len = scratchLen_;
    // Host side of BackSubstitution: swap buffers into the window, record
    // the outputs (exact lengths arrive with the completion, complete_solve).
    bool advanced = false;
    {
        std::lock_guard<std::mutex> g(res_->mu);
        recovered_.resize(m);
        ++decodeSerial_;
        PendingDecode& pd = res_->pend[slot];
        pd.serial = decodeSerial_;
        std::vector<Fix>& fixes = pd.fixes;
        fixes.clear();
        for (int ci = (int)m - 1; ci >= 0; --ci) {
            RecPacket* r = pr[ci];
            ColInfo& col = cols_[ci];
            DecSlot* o = col.original;
            // (a slab slot is not the slot's to give: the recovery packet
            // gets it only when owned)
            DevBuf old = o->inSlab ? DevBuf() : o->buf;
            o->inSlab = false;
            o->buf = r->buf;
            o->bytes = len[ci];
            o->column = col.column;
            o->header = 0;
            o->pending = true;
            o->pendSlot = slot;
            o->pendCi = (uint32_t)ci;
            r->buf = old;
            r->bytes = 0;
            SiameseOriginalPacket& out = recovered_[ci];
            out.PacketNum = col.column;
            out.DataBytes = 0;
            out.Data = nullptr;
            recoveredColumns_.push_back(col.column);
            advanced |= mark_got(col.column);
            fixes.push_back(Fix{o, o->buf.ptr, (uint32_t)ci, (unsigned)ci, len[ci]});
        }
        if (mirror_)   // (download_recovered's list: the drop-in API only)
            lastDecoded_ = fixes;
        publish_outputs();
        if (pd.held) {
            // a chained solve: its completion already arrived
            pd.held = false;
            if (pd.done && !mirror_)
                for (unsigned ci = 0; ci < m; ++ci)
                    fill_entry(pd, ci, recovered_[ci]);
        }
    }
    lastPendSlot_ = slot;

    if (!advanced) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    iterate_next_expected(region_.nextCheckStart);
    list_delete_before(nextExpected_);
    if (region_.nextCheckStart >= kRemoveThreshold)
        remove_elements();
    stats_[SiameseDecoderStats_SolveSuccessCount]++;
    return Siamese_Success;
}

// finish_chained's host side of BackSubstitution: as solve_publish and the
// apply_resolved that would follow it, the solve's lengths being known (its
// submission has completed): the window takes the recovered buffers with
// their exact lengths, the outputs are final.  A solve that flagged a corrupt
// length prefix goes the general way.
SiameseResult DecoderCore::publish_final(unsigned slot)
{
    const unsigned m = region_.lostCount;
    bool ready = false;
    {
        std::lock_guard<std::mutex> g(res_->mu);
        const PendingDecode& pd = res_->pend[slot];
        ready = pd.done && pd.words.size() > m && pd.words[0] == m;
    }
    if (!ready) {
        const SiameseResult res = solve_publish(slot);
        settle();
        return res;
    }
    const std::vector<RecPacket*>& pr = scratchRec_;
    bool advanced = false;
    {
        std::lock_guard<std::mutex> g(res_->mu);
        PendingDecode& pd = res_->pend[slot];
        recovered_.resize(m);
        ++decodeSerial_;
        for (int ci = (int)m - 1; ci >= 0; --ci) {
            RecPacket* r = pr[ci];
            ColInfo& col = cols_[ci];
            DecSlot* o = col.original;
            const uint32_t w = pd.words[1 + ci];
            const unsigned hdr = w >> 29, len = w & kSolveLengthMask;
            DevBuf old = o->inSlab ? DevBuf() : o->buf;
            o->inSlab = false;
            o->buf = r->buf;
            o->bytes = hdr + len;
            o->column = col.column;
            o->header = hdr;
            o->pending = false;
            r->buf = old;
            r->bytes = 0;
            SiameseOriginalPacket& out = recovered_[ci];
            out.PacketNum = col.column;
            out.DataBytes = len;
            out.Data = o->buf.ptr + hdr;
            recoveredColumns_.push_back(col.column);
            advanced |= mark_got(col.column);
        }
        publish_outputs();
        // (applied here, as apply_resolved would: its completion counted)
        pd.live = pd.done = pd.held = false;
        pd.fixes.clear();
    }
    pendingSolves_--;
    ++appliedCount_;
    lastPendSlot_ = slot;
    if (!advanced) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    iterate_next_expected(region_.nextCheckStart);
    list_delete_before(nextExpected_);
    if (region_.nextCheckStart >= kRemoveThreshold)
        remove_elements();
    stats_[SiameseDecoderStats_SolveSuccessCount]++;
    return Siamese_Success;
}

void DecoderCore::publish_outputs()
{
    res_->out = recovered_.data();
    res_->outCount = recovered_.size();
    res_->outSerial = decodeSerial_;
}

void DecoderCore::fill_entry(const PendingDecode& pd, unsigned ci, SiameseOriginalPacket& out)
{
    const unsigned okCount = pd.words[0];
    if (ci >= pd.m || ci + okCount < pd.m) {
        // not reached before a corrupt length prefix (reference :1142-1154)
        out.DataBytes = 0;
        out.Data = nullptr;
        return;
    }
    const uint32_t w = pd.words[1 + ci];
    out.DataBytes = w & kSolveLengthMask;
    out.Data = pd.fixes[pd.m - 1 - ci].buf + (w >> 29);
}

// Engine completer thread: the submission carrying the solve has completed.
void DecoderCore::complete_solve(Resolver& r, unsigned slot, const uint32_t* results)
{
    std::lock_guard<std::mutex> g(r.mu);
    PendingDecode& pd = r.pend[slot];
    pd.words.assign(results + pd.base, results + pd.base + pd.m + 1);
    for (const auto& t : pd.targets)
        fill_entry(pd, t.first, *t.second);
    pd.targets.clear();
    if (!r.orphan && !r.mirror && pd.serial == r.outSerial)
        for (unsigned ci = 0; ci < pd.m && ci < r.outCount; ++ci)
            fill_entry(pd, ci, r.out[ci]);
    pd.done = true;
    r.doneCount.fetch_add(1, std::memory_order_release);
}

// Owner thread: apply arrived completions to the decoder's own state.
void DecoderCore::apply_resolved()
{
    std::lock_guard<std::mutex> g(res_->mu);
    std::vector<PendingDecode>& pend = res_->pend;
    for (unsigned k = 0; k < pend.size(); ++k) {
        PendingDecode& pd = pend[k];
        if (!pd.live || !pd.done || pd.held)
            continue;
        const unsigned m = pd.m;
        const unsigned okCount = pd.words[0];
        if (okCount < m)
            disabled_ = true; // corrupt length prefix (reference :1142-1154)
        for (const Fix& f : pd.fixes) {
            const unsigned ci = f.outIndex;
            if (ci + okCount < m)
                continue; // not reached before the failure
            const uint32_t w = pd.words[1 + ci];
            const unsigned hdr = w >> 29;
            const unsigned len = w & kSolveLengthMask;
            DecSlot* s = f.slot;
            if (s->pending && s->buf.ptr == f.buf && s->pendSlot == k && s->pendCi == ci) {
                s->bytes = hdr + len;
                s->header = hdr;
                s->pending = false;
                if (mirror_ && s->host().size() < s->bytes)
                    s->host().resize(s->bytes);
            }
            if (mirror_ && pd.serial == decodeSerial_ && ci < recovered_.size()) {
                SiameseOriginalPacket& out = recovered_[ci];
                out.DataBytes = len;
                out.Data = s->host().data() + hdr;
            }
        }
        pd.live = false;
        pd.done = false;
        pendingSolves_--;
        ++appliedCount_;
    }
}

void DecoderCore::download_recovered()
{
    if (!mirror_)
        return;
    for (const Fix& f : lastDecoded_) {
        DecSlot* s = f.slot;
        s->host().resize(f.bound);
        eng_->download(s->host().data(), (uint64_t)(uintptr_t)f.buf, f.bound);
    }
    lastDecoded_.clear();
}

SiameseResult DecoderCore::get(SiameseOriginalPacket& packet)
{
    settle();
    if (dead())
        return Siamese_Disabled;
    const unsigned element = column_to_element(packet.PacketNum);
    if (element >= count_ || slot(element).bytes == 0) {
        packet.Data = nullptr;
        packet.DataBytes = 0;
        return Siamese_NeedMoreData;
    }
    if (slot(element).pending) {
        // Exact length still on the device: finish the outstanding work.
        // The drop-in API calls this under its shared instance lock, which a
        // detaching flush takes exclusively: it must flush outside the lock
        // (siamese_decoder_get does), so it gets kNeedsFlush back here.
        if (mirror_)
            return kNeedsFlush;
        if (!eng_->flush_and_sync())
            return Siamese_Disabled;
        settle();
        if (dead())
            return Siamese_Disabled;
    }
    DecSlot& s = slot(element);
    packet.Data = (mirror_ ? s.host().data() : s.buf.ptr) + s.header;
    packet.DataBytes = s.bytes - s.header;
    return Siamese_Success;
}

SiameseResult DecoderCore::get_range(unsigned firstNum, unsigned count, SiameseOriginalPacket* out, unsigned* got)
{
    *got = 0;
    // get() per packet, with the state checks made once and the window
    // walked slot by slot; a packet whose length is still on the device (or
    // anything else get() handles) goes through get() itself
    settle();
    const bool ok = !dead();
    unsigned e = column_to_element(firstNum);
    for (unsigned k = 0; k < count; ++k, e = (e + 1) % kColumnPeriod) {
        SiameseOriginalPacket& p = out[k];
        p.PacketNum = (firstNum + k) & SIAMESE_PACKET_NUM_MAX;
        if (ok && e < count_) {
            DecSlot& s = slot(e);
            if (s.bytes != 0 && !s.pending) {
                p.Data = (mirror_ ? s.host().data() : s.buf.ptr) + s.header;
                p.DataBytes = s.bytes - s.header;
                ++*got;
                continue;
            }
        }
        const SiameseResult r = get(p);
        if (r != Siamese_Success)
            return r;
        ++*got;
    }
    return Siamese_Success;
}

SiameseResult DecoderCore::decode_deferred(SiameseOriginalPacket* out, unsigned capacity, unsigned* countOut)
{
    settle();
    *countOut = 0;
    // room for any decode's outputs: a solve returns at most 255 packets
    // (kMaximumLossRecoveryCount), the single-recovery path what it holds
    if (capacity < kMaxLossRecovery || (hasRecovered_ && recovered_.size() > capacity))
        return Siamese_InvalidInput;
    SiameseOriginalPacket* p = nullptr;
    unsigned n = 0;
    const uint64_t serial = decodeSerial_;
    const SiameseResult r = decode(&p, &n);
    if (r != Siamese_Success)
        return r;
    std::copy(p, p + n, out);
    *countOut = n;
    if (decodeSerial_ != serial) {
        // a solve queued by this call: its lengths arrive with its completion
        std::lock_guard<std::mutex> g(res_->mu);
        PendingDecode& pd = res_->pend[lastPendSlot_];
        for (unsigned i = 0; i < n; ++i) {
            if (pd.done)
                fill_entry(pd, i, out[i]);
            else
                pd.targets.emplace_back(i, &out[i]);
        }
    }
    return Siamese_Success;
}

SiameseResult DecoderCore::get_deferred(SiameseOriginalPacket& packet)
{
    settle();
    if (dead())
        return Siamese_Disabled;
    const unsigned element = column_to_element(packet.PacketNum);
    if (element >= count_ || slot(element).bytes == 0) {
        packet.Data = nullptr;
        packet.DataBytes = 0;
        return Siamese_NeedMoreData;
    }
    DecSlot& s = slot(element);
    if (!s.pending) {
        packet.Data = (mirror_ ? s.host().data() : s.buf.ptr) + s.header;
        packet.DataBytes = s.bytes - s.header;
        return Siamese_Success;
    }
    std::lock_guard<std::mutex> g(res_->mu);
    PendingDecode& pd = res_->pend[s.pendSlot];
    if (pd.done) {
        fill_entry(pd, s.pendCi, packet);
    } else {
        packet.Data = nullptr;
        packet.DataBytes = 0;
        pd.targets.emplace_back(s.pendCi, &packet);
    }
    return Siamese_Success;
}

SiameseResult DecoderCore::stats(uint64_t* out, unsigned count)
{
    settle();
    if (count > SiameseDecoderStats_Count)
        count = SiameseDecoderStats_Count;
    uint64_t mem = 0;
    for (auto& sw : subwindows_) {
        mem += sw->slab.buf.cap;
        for (DecSlot& s : sw->slot)
            if (!s.inSlab)
                mem += s.buf.cap;
    }
    for (auto& lane : lanes_)
        for (Sum& s : lane)
            mem += s.d.buf.cap;
    for (RecPacket* r = head_; r; r = r->next)
        mem += r->buf.cap;
    stats_[SiameseDecoderStats_MemoryUsed] = mem;
    for (unsigned i = 0; i < count; ++i)
        out[i] = stats_[i];
    return Siamese_Success;
}

} // namespace sgpu
