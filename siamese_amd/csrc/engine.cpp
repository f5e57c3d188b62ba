// engine.cpp -- arena, programs and the asynchronous flush pipeline (see
// engine.h).
#include "engine.h"

#include <pthread.h>
#include "backend.h"
#include "codedef.h"
#include "pool.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>

// dispatch each exec phase's segments longest op list first (see launch_batch)
#ifndef SGPU_EXEC_LPT
#define SGPU_EXEC_LPT 1
#endif
// k_exec workgroups a launch aims for: a phase with more tiles than this
// gives each workgroup a run of its segment's tiles (one LDS-filling
// workgroup per CU: 256 CUs)
#ifndef SGPU_EXEC_GROUPS
#define SGPU_EXEC_GROUPS 256
#endif

namespace sgpu {

void EngineStats::add(const EngineStats& o)
{
    flushes += o.flushes;
    launches += o.launches;
    ops += o.ops;
    terms += o.terms;
    solves += o.solves;
    ingests += o.ingests;
    uploadBytes += o.uploadBytes;
    refOpBytes += o.refOpBytes;
    outBytes += o.outBytes;
    solveBytes += o.solveBytes;
    ldpcBytes += o.ldpcBytes;
    assembleNs += o.assembleNs;
    waitNs += o.waitNs;
    completeNs += o.completeNs;
    reclaimNs += o.reclaimNs;
    execLaunches += o.execLaunches;
    execUniqueBytes += o.execUniqueBytes;
    geJobs += o.geJobs;
    geChained += o.geChained;
    geRetried += o.geRetried;
}

namespace {

uint64_t now_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

inline size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

} // namespace

// ---------------------------------------------------------------------------
// ProgramBody

namespace {
std::mutex g_bodyMu;
std::vector<ProgramBody*> g_bodies;   // cleared bodies ready for reuse
} // namespace

ProgramBody* ProgramBody::get()
{
    {
        std::lock_guard<std::mutex> g(g_bodyMu);
        if (!g_bodies.empty()) {
            ProgramBody* b = g_bodies.back();
            g_bodies.pop_back();
            return b;
        }
    }
    return new ProgramBody;
}

void ProgramBody::put(ProgramBody* b)
{
    b->clear();
    std::lock_guard<std::mutex> g(g_bodyMu);
    if (g_bodies.size() < (1u << 15))
        g_bodies.push_back(b);
    else
        delete b;
}

void ProgramBody::clear()
{
    for (size_t k = 0; k < nsegs; ++k)
        segs[k].clear();
    nsegs = 0;
    resultWords = 0;
    nsolves = 0;   // (their vectors keep their capacity)
    nges = 0;
    callbacks.clear();
    keep.clear();
    rb.open = false;
    rb.win.clear();
    rb.updates.clear();
    rb.rows.clear();
    copies.clear();
    lcb.clear();
    gateOpen = false;
}

void ProgramBody::new_segment()
{
    rows_close();
    if (nsegs == segs.size())
        segs.emplace_back();
    segs[nsegs++].clear();
}

void ProgramBody::rows_open(uint32_t base, bool keepWindow)
{
    rows_close();
    if (nsegs == 0)
        new_segment();
    rb.open = true;
    rb.haveSums = false;
    rb.sumsVersion = 0;
    rb.readMask = 0;
    rb.cutMax = 0;
    rb.versioned = false;
    if (!keepWindow) {
        rb.base = base;
        rb.win.clear();
    }
    rb.updates.clear();
    for (int& u : rb.updateOf)
        u = -1;
    rb.rows.clear();
    rb.maxExtent = 0;
}

namespace {
// [a, a + an) and [b, b + bn) share a byte
inline bool overlaps(uint64_t a, uint64_t an, uint64_t b, uint64_t bn) { return a < b + bn && b < a + an; }
inline uint64_t lane_span(uint32_t n) { return ((uint64_t)n + 15) & ~(uint64_t)15; }
} // namespace

void ProgramBody::lc_seal()
{
    if (lcb.items.empty())
        return;
    Segment& s = segs[nsegs - 1];
    if (lcb.items.size() == 1) {
        // one combination: the plain op (all waves share its terms)
        const LcItem& it = lcb.items[0];
        GfOp op;
        std::memset(&op, 0, sizeof(op));
        op.dst = it.dst;
        op.n = it.n;
        op.valid = it.valid;
        op.kind = OP_LINCOMB;
        op.mix = it.mixLit & 0xff;
        op.termBegin = (uint32_t)s.terms.size();
        op.termCount = it.termCount;
        s.ops.push_back(op);
        s.terms.insert(s.terms.end(), lcb.terms.begin(), lcb.terms.end());
        const uint32_t litLen = (it.mixLit >> 8) & 0xff;
        if (litLen) {
            GfOp lo;
            std::memset(&lo, 0, sizeof(lo));
            lo.dst = it.dst;
            lo.n = it.litOffset;
            lo.valid = litLen;
            lo.kind = OP_LITERAL;
            std::memcpy(lo.lit, it.lit, litLen);
            s.ops.push_back(lo);
        }
        lcb.clear();
        return;
    }
    const uint32_t itemWords = (uint32_t)lcb.items.size() * kLcWords;
    for (LcItem& it : lcb.items)
        it.termStart += itemWords;   // (block-relative word of its first term)
    GfOp op;
    std::memset(&op, 0, sizeof(op));
    op.kind = OP_LINCOMBS;
    op.n = (uint32_t)lcb.items.size();
    op.termBegin = (uint32_t)(s.rowsData.size() / 16);
    op.termCount = itemWords + (uint32_t)lcb.terms.size();
    s.ops.push_back(op);
    const size_t at = s.rowsData.size();
    s.rowsData.resize(at + (size_t)op.termCount * 16);
    std::memcpy(s.rowsData.data() + at, lcb.items.data(), lcb.items.size() * sizeof(LcItem));
    std::memcpy(s.rowsData.data() + at + lcb.items.size() * sizeof(LcItem), lcb.terms.data(),
                lcb.terms.size() * sizeof(GfTerm));
    s.rowsWords += op.termCount;
    lcb.clear();
}

namespace {

using Span = ProgramBody::LcBuild::Span;

// does [lo, hi) meet a span of the disjoint sorted set v?
bool span_hits(const std::vector<Span>& v, uint64_t lo, uint64_t hi)
{
    const auto it = std::upper_bound(v.begin(), v.end(), lo,
                                     [](uint64_t x, const Span& sp) { return x < sp.hi; });
    return it != v.end() && it->lo < hi;
}

// v |= [lo, hi), keeping v disjoint and sorted
void span_add(std::vector<Span>& v, uint64_t lo, uint64_t hi)
{
    if (lo >= hi)
        return;
    auto first = std::lower_bound(v.begin(), v.end(), lo,
                                  [](const Span& sp, uint64_t x) { return sp.hi < x; });
    auto last = first;
    while (last != v.end() && last->lo <= hi) {
        lo = std::min(lo, last->lo);
        hi = std::max(hi, last->hi);
        ++last;
    }
    if (first == last) {
        v.insert(first, Span{lo, hi});
    } else {
        *first = Span{lo, hi};
        v.erase(first + 1, last);
    }
}

// bytes an item writes: its lanes and its footer literal
uint64_t lc_write_span(const LcItem& it)
{
    const uint32_t litEnd = it.litOffset + ((it.mixLit >> 8) & 0xff);
    return std::max<uint64_t>(lane_span(it.n), litEnd);
}

} // namespace

void ProgramBody::lc_absorb()
{
    // SIAMESE_AMD_LC_BATCH=0: every combination stays a plain op (A/B aid)
    static const bool enabled = [] {
        const char* v = std::getenv("SIAMESE_AMD_LC_BATCH");
        return !v || std::atoi(v) != 0;
    }();
    if (!enabled)
        return;
    Segment& s = segs[nsegs - 1];
    const GfOp op = s.ops.back();
    const GfTerm* t = s.terms.data() + op.termBegin;
    if (op.termCount > kLcMaxTerms) {
        // stays a plain op; the batch before it is sealed ahead of it
        s.ops.pop_back();
        lc_seal();
        s.ops.push_back(op);
        return;
    }
    // independent of every item of the open batch?  (writes: [dst,
    // align16(n)) and the literal; reads: the terms and dst's kept bytes)
    bool indep = lcb.items.size() < kLcMaxItems;
    const uint64_t w = lane_span(op.n);
    if (indep && !lcb.items.empty()) {
        // the items before the last: the span sets
        if (span_hits(lcb.writes, op.dst, op.dst + w) || span_hits(lcb.reads, op.dst, op.dst + w))
            indep = false;
        for (uint32_t k = 0; indep && k < op.termCount; ++k)
            if (span_hits(lcb.writes, t[k].src, t[k].src + lane_span(t[k].len)))
                indep = false;
        // the last item
        const LcItem& it = lcb.items.back();
        const uint64_t iw = lc_write_span(it);
        if (indep && overlaps(op.dst, w, it.dst, iw))
            indep = false;
        for (uint32_t k = 0; indep && k < op.termCount; ++k)
            if (overlaps(t[k].src, lane_span(t[k].len), it.dst, iw))
                indep = false;
        const GfTerm* u = lcb.terms.data() + it.termStart;
        for (uint32_t k = 0; indep && k < it.termCount; ++k)
            if (overlaps(u[k].src, lane_span(u[k].len), op.dst, w))
                indep = false;
    }
    // (its terms are the segment's last: move them out before a seal of a
    // single-item batch appends that item's terms to the segment)
    lcScratch.assign(t, t + op.termCount);
    s.terms.resize(op.termBegin);
    s.ops.pop_back();
    if (!indep) {
        lc_seal();
    } else if (!lcb.items.empty()) {
        // the last item joins the span sets (its literal can no longer grow)
        const LcItem& it = lcb.items.back();
        span_add(lcb.writes, it.dst, it.dst + lc_write_span(it));
        const GfTerm* u = lcb.terms.data() + it.termStart;
        for (uint32_t k = 0; k < it.termCount; ++k)
            span_add(lcb.reads, u[k].src, u[k].src + lane_span(u[k].len));
    }
    LcItem it;
    std::memset(&it, 0, sizeof(it));
    it.dst = op.dst;
    it.n = op.n;
    it.valid = op.valid;
    it.termStart = (uint32_t)lcb.terms.size();
    it.termCount = op.termCount;
    it.mixLit = op.mix & 0xff;
    lcb.items.push_back(it);
    lcb.terms.insert(lcb.terms.end(), lcScratch.begin(), lcScratch.end());
}

bool ProgramBody::lc_literal_fits(uint64_t at, uint32_t len) const
{
    // the literal's bytes must not be read or written by another item (the
    // items before the last: exactly the span sets)
    return !span_hits(lcb.writes, at, at + len) && !span_hits(lcb.reads, at, at + len);
}

void ProgramBody::rows_close()
{
    lc_seal();
    if (!copies.empty()) {
        // seal the open copy batch
        Segment& g = segs[nsegs - 1];
        GfOp op;
        std::memset(&op, 0, sizeof(op));
        op.kind = OP_COPIES;
        op.n = (uint32_t)copies.size();
        op.termBegin = (uint32_t)(g.rowsData.size() / 16);
        op.termCount = (uint32_t)copies.size() * kCopyWords;
        g.ops.push_back(op);
        const size_t at = g.rowsData.size();
        g.rowsData.resize(at + copies.size() * sizeof(CopyItem));
        std::memcpy(g.rowsData.data() + at, copies.data(), copies.size() * sizeof(CopyItem));
        g.rowsWords += op.termCount;
        copies.clear();
    }
    RowsBuild& b = rb;
    if (!b.open)
        return;
    b.open = false;
    if (b.rows.empty() && b.updates.empty())
        return;
    if (!b.haveSums)
        std::memset(b.sums, 0, sizeof(b.sums));
    Segment& s = segs[nsegs - 1];
    // wide rows: their LDPC picks run in k_ldpc (ops.h); the row reads the
    // two results as window entries appended after the snapshot (for this
    // block only: a batch opened with keepWindow continues the snapshot)
    const size_t winKept = b.win.size();
    for (RowItem& r : b.rows) {
        if (r.ldpcN < kLdpcSplitMin)
            continue;
        const uint32_t entry = (uint32_t)b.win.size();
        const uint32_t pairs = (r.ldpcN + kPairRate - 1) / kPairRate;
        s.wide.push_back(Segment::Wide{(uint32_t)s.ops.size(), entry, r.n, r.row, r.ldpcN, r.ldpcOff});
        s.wideItems += ((r.n + kLdpcTileBytes - 1) / kLdpcTileBytes) *
                       ((pairs + ldpc_pairs_per_item(r.n) - 1) / ldpc_pairs_per_item(r.n));
        s.wideBytes += 2 * (uint64_t)((r.n + kLdpcTileBytes - 1) / kLdpcTileBytes * kLdpcTileBytes);
        WinEntry z;
        std::memset(&z, 0, sizeof(z));
        b.win.push_back(z);   // (addresses patched at assembly)
        b.win.push_back(z);
        r.ldpcN = 0;
        r.ldpcOff = entry;
        r.mask0 |= kRowWide;
    }
    const uint32_t E = (uint32_t)b.win.size();
    const uint32_t U = (uint32_t)b.updates.size();
    const uint32_t R = (uint32_t)b.rows.size();
    const uint32_t words = kRowSums + E + U * kUpdateWords + R * kRowWords;
    // the executor stages window elements from the first one the batch reads
    // (updates, LDPC draws, wide rows' sums), not from the window's start
    uint32_t stageLo = E;
    for (const SumUpdate& u : b.updates)
        if (u.to > u.from)
            stageLo = std::min(stageLo, u.from);
    for (const RowItem& r : b.rows)
        if (r.ldpcN || (r.mask0 & kRowWide))
            stageLo = std::min(stageLo, r.ldpcOff);
    GfOp op;
    std::memset(&op, 0, sizeof(op));
    // (OP_ROWS has no dst of its own)
    op.dst = stageLo | (uint64_t)(b.versioned ? std::min<uint32_t>(R, kVersionRows) : 0u) << 32;
    op.kind = OP_ROWS;
    op.n = R;
    op.valid = E;
    op.mix = U;
    op.termBegin = (uint32_t)(s.rowsData.size() / 16);   // block offset in words
    op.termCount = words;
    s.ops.push_back(op);
    const size_t at = s.rowsData.size();
    s.rowsData.resize(at + (size_t)words * 16);
    uint8_t* w = s.rowsData.data() + at;
    std::memcpy(w, b.sums, sizeof(b.sums));
    w += sizeof(b.sums);
    std::memcpy(w, b.win.data(), (size_t)E * sizeof(WinEntry));
    w += (size_t)E * sizeof(WinEntry);
    std::memcpy(w, b.updates.data(), (size_t)U * sizeof(SumUpdate));
    w += (size_t)U * sizeof(SumUpdate);
    std::memcpy(w, b.rows.data(), (size_t)R * sizeof(RowItem));
    b.win.resize(winKept);
    s.rowsWords += words;
    if (b.maxExtent > s.maxExtent)
        s.maxExtent = b.maxExtent;
}

// ---------------------------------------------------------------------------
// Program

Program::~Program()
{
    if (!shard_) {
        if (b_)
            ProgramBody::put(b_);
        return;
    }
    // The instance goes away with work still queued (e.g. an encoder freed
    // right after its last recovery packet was handed to a decoder, whose
    // copy op lives in this program).  The queued ops still run: hand the
    // body to an orphan program the next submission takes and deletes.  The
    // buffers they touch were released by the instance and are not reused
    // before that submission completes.
    Program* orphan = new Program(eng_, group_ | 2);   // bit 1: delete when submitted
    orphan->shard_ = shard_;
    orphan->b_ = b_;
    b_ = nullptr;
    std::lock_guard<std::mutex> g(shard_->mu);
    auto it = std::find(shard_->dirty.begin(), shard_->dirty.end(), this);
    if (it != shard_->dirty.end())
        *it = orphan;
}

void Program::attach()
{
    if (!b_)
        b_ = ProgramBody::get();
    b_->group = group_ & 1;
    Shard& s = eng_->shard();
    shard_ = &s;
    std::lock_guard<std::mutex> g(s.mu);
    s.dirty.push_back(this);
}

void Program::lc_begin(uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix)
{
    touch();
    if (b_->rb.open || !b_->copies.empty()) {
        // (an open OP_LINCOMBS batch stays open: lc_end decides)
        b_->lc_seal();
        b_->rows_close();
    }
    if (b_->nsegs == 0)
        b_->new_segment();
    ProgramBody::Segment& s = b_->segs[b_->nsegs - 1];
    GfOp op;
    op.dst = dst;
    op.n = n;
    op.valid = valid < n ? valid : n;
    op.kind = OP_LINCOMB;
    op.mix = mix;
    op.termBegin = (uint32_t)s.terms.size();
    op.termCount = 0;
    s.ops.push_back(op);
}

void Program::lc_end()
{
    ProgramBody::Segment& s = b_->segs[b_->nsegs - 1];
    GfOp& op = s.ops.back();
    // An op that keeps all of dst and adds nothing is a no-op.
    if (op.termCount == 0 && op.valid >= op.n) {
        s.ops.pop_back();
        return;
    }
    if (op.n > s.maxExtent)
        s.maxExtent = op.n;
    b_->lc_absorb();
}

void Program::add_mem(uint64_t dst, uint64_t src, uint32_t n)
{
    if (n == 0)
        return;
    lc_begin(dst, n, n);
    lc_term(src, n, 1);
    lc_end();
}

void Program::muladd_mem(uint64_t dst, uint8_t y, uint64_t src, uint32_t n)
{
    if (n == 0 || y == 0)
        return;
    lc_begin(dst, n, n);
    lc_term(src, n, y);
    lc_end();
}

void Program::mul_mem(uint64_t dst, uint64_t src, uint8_t y, uint32_t n)
{
    if (n == 0)
        return;
    lc_begin(dst, n, 0);
    lc_term(src, n, y);
    lc_end();
}

void Program::zero(uint64_t dst, uint32_t n)
{
    if (n == 0)
        return;
    lc_begin(dst, n, 0);
    lc_end();
}

void Program::literal(uint64_t dst, uint32_t offset, const uint8_t* bytes, uint32_t len)
{
    if (len == 0)
        return;
    touch();
    if (!b_->lcb.items.empty()) {
        // a footer right after its combination joins that batch item
        LcItem& it = b_->lcb.items.back();
        if (it.dst == dst && (it.mixLit >> 8) == 0 && len <= 8 && b_->lc_literal_fits(dst + offset, len)) {
            it.mixLit |= len << 8;
            it.litOffset = offset;
            std::memcpy(it.lit, bytes, len);
            ProgramBody::Segment& s = b_->segs[b_->nsegs - 1];
            if (offset + len > s.maxExtent)
                s.maxExtent = offset + len;
            return;
        }
    }
    b_->rows_close();
    if (b_->nsegs == 0)
        b_->new_segment();
    ProgramBody::Segment& s = b_->segs[b_->nsegs - 1];
    GfOp op;
    std::memset(&op, 0, sizeof(op));
    op.dst = dst;
    op.n = offset;
    op.valid = len;
    op.kind = OP_LITERAL;
    std::memcpy(op.lit, bytes, len);
    s.ops.push_back(op);
    if (offset + len > s.maxExtent)
        s.maxExtent = offset + len;
}

void Program::ingest_host(const DevBuf& dst, const void* data, uint32_t bytes, const uint8_t* hdr,
                          uint32_t hdrLen)
{
    eng_->stage_host_ingest(dst, data, bytes, hdr, hdrLen);
}

void Program::ingest_device(const DevBuf& dst, uint64_t src, uint32_t bytes, const uint8_t* hdr,
                            uint32_t hdrLen)
{
    ingest_run(dst.addr(), 0, src, 0, 1, bytes, hdr, hdrLen);
}

void Program::ingest_run(uint64_t dst, uint32_t dstStride, uint64_t src, uint32_t srcStride, uint32_t count,
                         uint32_t bytes, const uint8_t* hdr, uint32_t hdrLen)
{
    IngestDesc d;
    std::memset(&d, 0, sizeof(d));
    d.dst = dst;
    d.src = src;
    d.bytes = bytes;
    d.hdrLen = hdrLen;
    d.count = count;
    d.srcStride = count > 1 ? srcStride : 0;
    d.dstStride = count > 1 ? dstStride : 0;
    std::memcpy(d.hdr, hdr, hdrLen < 8 ? hdrLen : 8);
    eng_->add_ingest(d, -1);
}

uint32_t Program::solve(const std::vector<SolveRow>& rows, const uint8_t* coef, uint32_t maxBytes)
{
    SolveRow* r = nullptr;
    uint8_t* c = nullptr;
    solve_reserve((unsigned)rows.size(), &r, &c);
    std::memcpy(r, rows.data(), rows.size() * sizeof(SolveRow));
    std::memcpy(c, coef, rows.size() * rows.size());
    return solve_commit(maxBytes);
}

void Program::solve_reserve(unsigned m, SolveRow** rows, uint8_t** coef)
{
    touch();
    if (b_->nsegs == 0)
        b_->new_segment(); // the segment preceding this solve
    if (b_->nsolves == b_->solves.size())
        b_->solves.emplace_back();
    ProgramBody::PendingSolve& ps = b_->solves[b_->nsolves];
    ps.rows.resize(m);
    ps.coef.resize((size_t)m * m);
    *rows = ps.rows.data();
    *coef = ps.coef.data();
}

uint32_t Program::solve_commit(uint32_t maxBytes, uint32_t gateWord)
{
    ProgramBody::PendingSolve& ps = b_->solves[b_->nsolves++];
    const size_t m = ps.rows.size();
    // each row's first 16 bytes as the solve will find them, for the length
    // prefix pass every tile of the solve runs (SolveDesc.head): one copy
    // batch, built in place
    DevBuf head = eng_->alloc((uint32_t)m * 16u);
    if (head) {
        if (b_->copies.empty()) {
            b_->rows_close();
            if (b_->nsegs == 0)
                b_->new_segment();
        }
        std::vector<CopyItem>& cp = b_->copies;
        size_t at = cp.size();
        cp.resize(at + m);
        uint32_t ext = 0;
        for (size_t i = 0; i < m; ++i) {
            const uint32_t len = std::min<uint32_t>(16u, ps.rows[i].initBytes);
            if (len == 0)
                continue;   // (as copy(): nothing to move)
            CopyItem& c = cp[at++];
            std::memset(&c, 0, sizeof(c));
            c.dst = head.addr() + i * 16;
            c.src = ps.rows[i].buf;
            c.len = len;
            ext = std::max(ext, len);
        }
        cp.resize(at);
        ProgramBody::Segment& g = b_->segs[b_->nsegs - 1];
        if (ext > g.maxExtent)
            g.maxExtent = ext;
        b_->rows_close();   // (seal the copy batch into this segment)
    }
    std::memset(&ps.desc, 0, sizeof(ps.desc));
    ps.desc.head = head.addr();
    eng_->release(head);   // (reused only after this submission completes)
    ps.desc.m = (uint32_t)m;
    ps.desc.maxBytes = maxBytes;
    ps.desc.gate = gateWord;
    if (gateWord && b_->nges) {
        ProgramBody::PendingGe& g = b_->ges[b_->nges - 1];
        g.solve = (uint32_t)(b_->nsolves - 1);
    }
    ps.desc.result = b_->resultWords;
    b_->resultWords += ps.desc.m + 2;
    const uint32_t r = ps.desc.result;
    b_->new_segment(); // ops after the solve go to the next segment
    return r;
}

void Program::gate_begin(uint32_t word)
{
    touch();
    b_->rows_close();   // (ops queued before stay ungated)
    if (b_->nsegs == 0)
        b_->new_segment();
    b_->gateOpen = true;
    b_->gateSeg = b_->nsegs - 1;
    b_->gateOp = (uint32_t)b_->segs[b_->nsegs - 1].ops.size();
    b_->gateWord = word;
}

void Program::gate_end()
{
    if (!b_ || !b_->gateOpen)
        return;
    b_->rows_close();
    b_->gateOpen = false;
    ProgramBody::Segment& s = b_->segs[b_->gateSeg];
    if (b_->gateSeg + 1 == b_->nsegs && s.ops.size() > b_->gateOp)
        s.gates.push_back(ProgramBody::Segment::Gate{b_->gateOp, (uint32_t)s.ops.size(), b_->gateWord});
}

uint8_t* Program::ge_job(unsigned rows, unsigned cols, unsigned pickLen, uint32_t* resultWord, bool chained)
{
    touch();
    if (b_->nges == b_->ges.size())
        b_->ges.emplace_back();
    ProgramBody::PendingGe& g = b_->ges[b_->nges++];
    g.rows = (uint16_t)rows;
    g.cols = (uint16_t)cols;
    g.pickLen = pickLen;
    g.result = b_->resultWords;
    g.chained = chained;
    g.solve = 0;
    b_->resultWords += ge_result_words(rows, cols, chained);
    g.in.resize(ge_input_bytes(rows, cols, pickLen));
    *resultWord = g.result;
    return g.in.data();
}

void Program::on_complete(Completion fn)
{
    touch();
    b_->callbacks.push_back(std::move(fn));
}

void Program::on_complete(std::shared_ptr<void> keep, Completion fn)
{
    touch();
    b_->keep.push_back(std::move(keep));
    b_->callbacks.push_back(std::move(fn));
}

// ---- Siamese row batches ---------------------------------------------------

WinEntry* Program::rows_window(uint32_t lo, uint32_t hi, uint32_t* from)
{
    touch();
    ProgramBody::RowsBuild& b = b_->rb;
    if (!b.open || lo < b.base)
        rows_open(lo, false);
    const uint32_t end = b.base + (uint32_t)b.win.size();
    if (hi <= end) {
        *from = hi;
        return nullptr;
    }
    *from = end;
    b.win.resize(hi - b.base);
    return b.win.data() + (end - b.base);
}

void Program::rows_update(unsigned k, uint64_t dst, uint32_t n, uint32_t valid, unsigned s,
                          uint32_t fromElement, uint32_t toElement)
{
    ProgramBody::RowsBuild& b = b_->rb;
    // A row of this batch already read sum k: the update may join the batch
    // only if it extends the sum those rows read (same buffer, keeping every
    // byte they saw), so each row can take back what was folded in after it
    // (RowItem.cutoff).  A restarted or moved sum starts a new batch, whose
    // rows run after this batch's rows.
    // Rows that read the sum before the update take its elements back out
    // (ops.h RowItem), so only short extensions join (a streaming encoder's
    // few new originals per row; not a decoder row whose range ends far past
    // the previous row's), into a batch of fewer than kVersionRows rows.
    if (b.readMask >> k & 1) {
        const WinEntry& seen = b.sums[k];
        if (seen.src != dst || valid < seen.len || toElement - fromElement > kVersionMaxSpan ||
            b.rows.size() >= kVersionRows)
            rows_open(b.base, true);
        else
            b.versioned = true;
    }
    const uint32_t from = fromElement - b.base, to = toElement - b.base;
    int& ui = b.updateOf[k];
    if (ui >= 0) {
        SumUpdate& u = b.updates[ui];
        const uint64_t d = ((uint64_t)u.dstHi << 32) | u.dstLo;
        if (d == dst && (u.to == from || from == to)) {
            // continue the same sum: one update over the joined element range
            if (from != to)
                u.to = to;
            if (n > u.n)
                u.n = n;
            if (n > b.maxExtent)
                b.maxExtent = n;
            return;
        }
        // a different buffer (the sum grew) or a gap: a fresh batch keeps
        // the two updates in order
        rows_open(b.base, true);
    }
    SumUpdate u;
    std::memset(&u, 0, sizeof(u));
    u.dstLo = (uint32_t)dst;
    u.dstHi = (uint32_t)(dst >> 32);
    u.n = n;
    u.valid = valid < n ? valid : n;
    u.s = s;
    u.from = from;
    u.to = to < from ? from : to;
    u.sum = k;   // (the executor refreshes that sum's stage slot from the update)
    b.updateOf[k] = (int)b.updates.size();
    b.updates.push_back(u);
    if (n > b.maxExtent)
        b.maxExtent = n;
}

uint64_t Program::next_table_version()
{
    static std::atomic<uint64_t> next{1};
    return next.fetch_add(1, std::memory_order_relaxed);
}

void Program::rows_row(const WinEntry* sums, uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix,
                       uint32_t mask0, uint32_t mask1, unsigned row, uint32_t ldpcN,
                       uint32_t ldpcFirst, uint32_t cutoff, const uint8_t* lit, uint32_t litLen,
                       uint64_t sumsVersion)
{
    ProgramBody::RowsBuild& b = b_->rb;
    // (the batch already holds this very table: nothing to compare or copy)
    const bool unchanged = sumsVersion != 0 && b.haveSums && b.sumsVersion == sumsVersion;
    // (a row whose cutoff is below an earlier row's reads sums folded past
    // its own cutoff: it starts a batch after every update so far; a
    // versioned batch takes at most kVersionRows rows)
    // The batch's sums table: entries an earlier row read must be this row's
    // too; an entry no row has read yet takes this row's value (a sum brought
    // up to date for this row: its update joined the batch, and the rows
    // before do not read it), so consecutive rows over one window share a
    // batch while the sums fill in.
    bool same = true;
    if (b.haveSums && !unchanged)
        for (uint32_t r = b.readMask; r; r &= r - 1) {
            const unsigned k = (unsigned)__builtin_ctz(r);
            if (std::memcmp(&b.sums[k], &sums[k], sizeof(WinEntry)) != 0) {
                same = false;
                break;
            }
        }
    if (!same || cutoff < b.cutMax || (b.versioned && b.rows.size() >= kVersionRows))
        rows_open(b.base, true);
    b.cutMax = std::max(b.cutMax, cutoff);
    if (!(unchanged && b.haveSums))   // (a batch opened just above copies)
        std::memcpy(b.sums, sums, sizeof(b.sums));
    b.haveSums = true;
    b.sumsVersion = sumsVersion;
    RowItem r;
    std::memset(&r, 0, sizeof(r));
    r.dst = dst;
    r.n = n;
    r.valid = valid < n ? valid : n;
    r.mask0 = mask0 | (litLen << 24);
    r.mask1 = mask1 | ((uint32_t)mix << 24);
    r.row = row;
    r.ldpcN = ldpcN;
    r.ldpcOff = ldpcFirst - b.base;
    r.cutoff = cutoff - b.base;
    if (litLen)
        std::memcpy(r.lit, lit, litLen);
    b.rows.push_back(r);
    b.readMask |= mask0 | mask1;
    if (n + litLen > b.maxExtent)
        b.maxExtent = n + litLen;
}

void Program::copy(uint64_t dst, uint64_t src, uint32_t len)
{
    if (len == 0)
        return;
    touch();
    if (b_->copies.empty()) {
        b_->rows_close();
        if (b_->nsegs == 0)
            b_->new_segment();
    }
    CopyItem c;
    std::memset(&c, 0, sizeof(c));
    c.dst = dst;
    c.src = src;
    c.len = len;
    b_->copies.push_back(c);
    ProgramBody::Segment& g = b_->segs[b_->nsegs - 1];
    if (len > g.maxExtent)
        g.maxExtent = len;
}

// ---------------------------------------------------------------------------
// Shard queues

bool Shard::Queues::empty() const
{
    if (!ingest.empty() || !downloads.empty())
        return false;
    for (const auto& r : released)
        if (!r.empty())
            return false;
    return true;
}

void Shard::Queues::clear()
{
    ingest.clear();
    hostStage.clear();
    downloads.clear();
    maxIngest = 0;
    pairCursor = 0;
    for (auto& r : released)
        r.clear();
}

// ---------------------------------------------------------------------------
// Engine: shards, arena, statistics

Engine* Engine::global()
{
    static Engine e;
    return &e;
}

Engine::~Engine() { stop_threads(); }

bool Engine::init(int device, const char** err)
{
    if (ready_)
        return true;
    if (!be_init(device, err))
        return false;
    start_threads();
    ready_ = true;
    return true;
}

Shard& Engine::shard()
{
    thread_local Engine* owner = nullptr;
    thread_local Shard* mine = nullptr;
    if (owner != this) {
        std::lock_guard<std::mutex> g(shardsMu_);
        shards_.emplace_back(new Shard);
        mine = shards_.back().get();
        owner = this;
    }
    return *mine;
}

WorkerPool& Engine::pool()
{
    static std::mutex m;
    std::lock_guard<std::mutex> g(m);
    if (!pool_)
        pool_.reset(new WorkerPool(WorkerPool::default_threads(), WorkerPool::shared_nice(), "sgpu-step"));
    return *pool_;
}

void Engine::account(uint64_t opBytes, uint64_t outBytes, bool inSolve)
{
    EngineStats& s = shard().stats;
    s.refOpBytes += opBytes;
    s.outBytes += outBytes;
    if (inSolve)
        s.solveBytes += opBytes + outBytes;
}

EngineStats Engine::stats() const
{
    EngineStats t;
    {
        std::lock_guard<std::mutex> g(const_cast<std::mutex&>(statsMu_));
        t = flushStats_;
    }
    std::lock_guard<std::mutex> g(shardsMu_);
    for (const auto& s : shards_)
        t.add(s->stats);
    return t;
}

uint64_t Engine::bytes_in_use() const
{
    int64_t t = 0;
    std::lock_guard<std::mutex> g(shardsMu_);
    for (const auto& s : shards_)
        t += s->inUse;
    return (uint64_t)t;
}

uint32_t round_cap(uint32_t bytes)
{
    if (bytes < 64)
        return 64;
    if (bytes <= 4096)
        return (bytes + 63) & ~63u;
    if (bytes <= 131072)
        return (bytes + 1023) & ~1023u;
    return (bytes + 65535) & ~65535u;
}

namespace {

size_t cap_class(uint32_t cap)
{
    if (cap <= 4096)
        return cap / 64 - 1;                 // 0..63
    if (cap <= 131072)
        return 64 + cap / 1024 - 5;          // 64..187
    return 188 + cap / 65536 - 3;
}

constexpr size_t kChunkBytes = 64u << 20;    // one hipMalloc
constexpr size_t kRegionBytes = 4u << 20;    // a shard's bump region
constexpr size_t kMagazine = 512;            // buffers cut per refill at most
constexpr size_t kMaxMagazine = 512;         // buffers per depot magazine at most (bounds what a shard hoards)
constexpr size_t kRefillBytes = 1u << 20;    // bytes carved per refill

} // namespace

uint8_t* Engine::carve_region(size_t bytes)
{
    std::lock_guard<std::mutex> g(arenaMu_);
    if (bytes > kChunkBytes / 4) {
        arenaBytes_ += bytes;
        return (uint8_t*)be_dev_alloc(bytes);
    }
    if (chunks_.empty() || chunks_.back().used + bytes > chunks_.back().size) {
        if (!spare_.empty()) {
            // a chunk reserved ahead (reserve()): no hipMalloc here
            chunks_.push_back(spare_.back());
            spare_.pop_back();
        } else {
            uint8_t* base = (uint8_t*)be_dev_alloc(kChunkBytes);
            if (!base)
                return nullptr;
            arenaBytes_ += kChunkBytes;
            chunks_.push_back(Chunk{base, kChunkBytes, 0});
        }
    }
    Chunk& c = chunks_.back();
    uint8_t* p = c.base + c.used;
    c.used += bytes;
    return p;
}

bool Engine::reserve(size_t bytes)
{
    std::lock_guard<std::mutex> g(arenaMu_);
    size_t have = 0;
    for (const Chunk& c : spare_)
        have += c.size;
    while (have < bytes) {
        uint8_t* base = (uint8_t*)be_dev_alloc(kChunkBytes);
        if (!base)
            return false;
        arenaBytes_ += kChunkBytes;
        spare_.push_back(Chunk{base, kChunkBytes, 0});
        have += kChunkBytes;
    }
    return true;
}

// Refill shard s's empty list of class `cls`: a magazine of buffers a
// completed submission returned, otherwise fresh buffers cut from the shard's
// bump region.
bool Engine::refill(Shard& s, size_t cls, uint32_t cap)
{
    std::vector<uint8_t*>& list = s.freeLists[cls];
    {
        // the newest magazine whose submission reads as done (the completer
        // files a submission's magazines just before it publishes the ticket)
        const uint64_t done = doneSeen_.load(std::memory_order_acquire);
        std::lock_guard<std::mutex> g(depotMu_);
        if (cls < depot_.size()) {
            auto& mags = depot_[cls];
            for (size_t k = mags.size(); k-- > 0;) {
                if (mags[k].ticket > done)
                    continue;
                list.swap(mags[k].bufs);
                mags.erase(mags.begin() + (long)k);
                if (!list.empty())
                    return true;
                break;
            }
        }
    }
    if (cap > kRegionBytes / 4) {
        uint8_t* p = carve_region(cap);
        if (!p)
            return false;
        list.push_back(p);
        return true;
    }
    const size_t want = std::max<size_t>(1, std::min<size_t>(kMagazine, kRefillBytes / cap));
    for (size_t k = 0; k < want; ++k) {
        if (s.bumpLeft < cap) {
            if (k > 0)
                break;
            uint8_t* r = carve_region(kRegionBytes);
            if (!r)
                return false;
            s.bump = r;           // the rest of the old region is abandoned (< cap)
            s.bumpLeft = kRegionBytes;
        }
        list.push_back(s.bump);
        s.bump += cap;
        s.bumpLeft -= cap;
    }
    return true;
}

DevBuf Engine::alloc(uint32_t bytes)
{
    DevBuf b;
    const uint32_t cap = round_cap(bytes);
    Shard& s = shard();
    const size_t cls = cap_class(cap);
    if (cls >= s.freeLists.size())
        s.freeLists.resize(cls + 1);
    if (s.freeLists[cls].empty() && !refill(s, cls, cap))
        return DevBuf();
    b.ptr = s.freeLists[cls].back();
    s.freeLists[cls].pop_back();
    b.cap = cap;
    s.inUse += cap;
    return b;
}


DevBuf Engine::slab_slot(Slab& sl, unsigned bit, uint32_t need, bool* failed)
{
    *failed = false;
    if (!sl.buf) {
        // slots of one MTU-sized class at least: a subwindow of small and
        // mixed-size datagrams still shares one slab
        constexpr uint32_t kMinSlot = 1408;
        const uint32_t stride = round_cap(std::max(need, kMinSlot));
        if ((uint64_t)stride * kSubwindow > 0xffffffffu)
            return DevBuf();
        sl.buf = alloc(stride * kSubwindow);
        if (!sl.buf) {
            *failed = true;
            return DevBuf();
        }
        sl.stride = stride;
        sl.used = 0;
    }
    if (need > sl.stride || (sl.used >> bit & 1u))
        return DevBuf();
    sl.used |= 1ull << bit;
    DevBuf b;
    b.ptr = sl.buf.ptr + (size_t)bit * sl.stride;
    b.cap = sl.stride;
    return b;
}

void Engine::release(DevBuf& b)
{
    if (b.ptr) {
        Shard& s = shard();
        const size_t cls = cap_class(b.cap);
        if (cls >= s.q.released.size())
            s.q.released.resize(cls + 1);
        s.q.released[cls].push_back(b.ptr);
        s.inUse -= b.cap;
    }
    b = DevBuf();
}

void Engine::download(void* hostDst, uint64_t devSrc, uint32_t bytes)
{
    if (bytes)
        shard().q.downloads.push_back(Shard::Download{hostDst, devSrc, bytes});
}

void Engine::stage_host_ingest(const DevBuf& dst, const void* data, uint32_t bytes,
                               const uint8_t* hdr, uint32_t hdrLen)
{
    // Stage hdr || data contiguously so the device copy is aligned.
    Shard& s = shard();
    const size_t off = (s.q.hostStage.size() + 15) & ~(size_t)15;
    s.q.hostStage.resize(off + hdrLen + bytes);
    std::memcpy(s.q.hostStage.data() + off, hdr, hdrLen);
    std::memcpy(s.q.hostStage.data() + off + hdrLen, data, bytes);
    IngestDesc d;
    std::memset(&d, 0, sizeof(d));
    d.dst = dst.addr();
    d.src = 0;
    d.bytes = hdrLen + bytes;
    d.hdrLen = 0;
    s.q.ingest.push_back(Shard::IngestRec{d, (int64_t)off});
    s.q.maxIngest = std::max(s.q.maxIngest, d.bytes);
}

namespace {

inline bool same_symbols(const IngestDesc& a, const IngestDesc& b)
{
    return a.bytes == b.bytes && a.hdrLen == b.hdrLen && std::memcmp(a.hdr, b.hdr, sizeof(a.hdr)) == 0;
}

inline uint32_t run_count(const IngestDesc& d)
{
    return d.count ? d.count : 1u;
}

/// Stride that takes `from` to `to` in one step (0: none fits 32 bits)
inline uint32_t step_of(uint64_t from, uint64_t to)
{
    return to > from && to - from <= 0xffffffffu ? (uint32_t)(to - from) : 0u;
}

/// Append run b to run a when b's symbols continue a's (same shape, same
/// strides, second destinations on one base); true if merged.
bool extend_run(IngestDesc& a, const IngestDesc& b)
{
    const uint32_t na = run_count(a), nb = run_count(b);
    if (!same_symbols(a, b) || na + nb > kIngestRunMax)
        return false;
    uint32_t ss = a.srcStride, ds = a.dstStride;
    if (na == 1) {   // a's strides are fixed by b's first symbol
        ss = step_of(a.src, b.src);
        ds = step_of(a.dst, b.dst);
        if (!ss || !ds)
            return false;
    }
    if (nb > 1 && (b.srcStride != ss || b.dstStride != ds))
        return false;
    if (b.src != a.src + (uint64_t)na * ss || b.dst != a.dst + (uint64_t)na * ds)
        return false;
    uint64_t base2 = a.dst2;
    if (b.dst2Mask) {
        const uint64_t want = b.dst2 - (uint64_t)na * ds;   // b's second base seen from a's symbol 0
        if (a.dst2Mask && want != a.dst2)
            return false;
        base2 = want;
    }
    a.srcStride = ss;
    a.dstStride = ds;
    a.dst2 = base2;
    a.dst2Mask |= b.dst2Mask << na;
    a.count = na + nb;
    return true;
}

} // namespace

void Engine::add_ingest(const IngestDesc& d, int64_t hostStageOffset)
{
    Shard::Queues& q = shard().q;
    // SIAMESE_AMD_INGEST_PAIRS=0 keeps an encoder's and a decoder's ingest of
    // one original apart (A/B aid)
    static const bool pairs = [] {
        const char* v = std::getenv("SIAMESE_AMD_INGEST_PAIRS");
        return !v || std::atoi(v) != 0;
    }();
    if (hostStageOffset < 0 && !q.ingest.empty()) {
        // The same device symbols as a recent run's (an encoder and then its
        // decoder taking in the same originals): the decoder's destinations
        // become that run's second destinations, the source read once.  The
        // run keeps one base for them; its mask says which symbols have one.
        // (The search looks at the last few runs and at the one matched last:
        // a decoder's runs follow its encoder's run by run.)
        if (pairs && d.dst2Mask == 0) {
            auto try_pair = [&](Shard::IngestRec& e) {
                if (e.hostOffset >= 0 || !same_symbols(e.d, d))
                    return false;
                const uint32_t n = run_count(e.d), c = run_count(d);
                const uint32_t ss = n > 1 ? e.d.srcStride : 0;
                uint32_t k;
                if (d.src == e.d.src)
                    k = 0;
                else if (ss && d.src > e.d.src && (d.src - e.d.src) % ss == 0 && (d.src - e.d.src) / ss < n)
                    k = (uint32_t)((d.src - e.d.src) / ss);
                else
                    return false;
                if (k + c > n || (c > 1 && (d.srcStride != ss || d.dstStride != e.d.dstStride)))
                    return false;   // (a run both sides must step through alike)
                const uint64_t base = d.dst - (uint64_t)k * e.d.dstStride;
                const uint64_t bits = (c >= 64 ? ~0ull : ((1ull << c) - 1)) << k;
                if (e.d.dst2Mask && (e.d.dst2 != base || (e.d.dst2Mask & bits)))
                    return false;
                e.d.dst2 = base;
                e.d.dst2Mask |= bits;
                return true;
            };
            const size_t sz = q.ingest.size();
            for (size_t i = q.pairCursor; i < sz && i < q.pairCursor + 8; ++i)
                if (try_pair(q.ingest[i])) {
                    q.pairCursor = i;
                    return;
                }
            const size_t lo = sz > 8 ? sz - 8 : 0;
            for (size_t i = sz; i-- > lo;)
                if (i >= q.pairCursor + 8 && try_pair(q.ingest[i])) {
                    q.pairCursor = i;
                    return;
                }
        }
        // the next symbols of the last run (consecutive slab slots from
        // consecutive device originals): one descriptor grows
        Shard::IngestRec& last = q.ingest.back();
        if (last.hostOffset < 0 && extend_run(last.d, d))
            return;
    }
    q.ingest.push_back(Shard::IngestRec{d, hostStageOffset});
    q.maxIngest = std::max(q.maxIngest, d.bytes + d.hdrLen);
}

bool Engine::pending() const
{
    std::lock_guard<std::mutex> g(shardsMu_);
    for (const auto& s : shards_)
        if (!s->dirty.empty() || !s->q.empty())
            return true;
    return false;
}

void Engine::ensure_up(XferSet& x, size_t bytes)
{
    if (bytes <= x.upCap)
        return;
    size_t cap = x.upCap ? x.upCap : (1u << 20);
    while (cap < bytes)
        cap *= 2;
    if (x.upHost)
        be_host_free(x.upHost);
    if (x.upDev)
        be_dev_free(x.upDev);
    x.upHost = (uint8_t*)be_host_alloc_mapped(cap);
    x.upDev = (uint8_t*)be_dev_alloc(cap);
    x.upHostDev = x.upHost ? (uint8_t*)be_host_device_ptr(x.upHost) : nullptr;
    x.upCap = cap;
}

void Engine::ensure_wide(XferSet& x, size_t bytes)
{
    if (bytes <= x.wideCap)
        return;
    size_t cap = x.wideCap ? x.wideCap : (1u << 20);
    while (cap < bytes)
        cap *= 2;
    if (x.wideDev)
        be_dev_free(x.wideDev);
    x.wideDev = (uint8_t*)be_dev_alloc(cap);
    x.wideCap = cap;
}

void Engine::ensure_solve(XferSet& x, size_t bytes)
{
    if (bytes <= x.solveCap)
        return;
    size_t cap = x.solveCap ? x.solveCap : (4u << 20);
    while (cap < bytes)
        cap *= 2;
    if (x.solveDev)
        be_dev_free(x.solveDev);
    x.solveDev = (uint8_t*)be_dev_alloc(cap);
    x.solveCap = cap;
}

void Engine::ensure_down(XferSet& x, size_t bytes)
{
    if (bytes <= x.downCap)
        return;
    size_t cap = x.downCap ? x.downCap : (1u << 20);
    while (cap < bytes)
        cap *= 2;
    if (x.downHost)
        be_host_free(x.downHost);
    if (x.downDev)
        be_dev_free(x.downDev);
    x.downHost = (uint8_t*)be_host_alloc_mapped(cap);
    x.downDev = (uint8_t*)be_dev_alloc(cap);
    x.downHostDev = x.downHost ? (uint8_t*)be_host_device_ptr(x.downHost) : nullptr;
    x.downCap = cap;
    x.acctZero = true;
    x.acctPrev[0] = x.acctPrev[1] = x.acctPrev[2] = x.acctPrev[3] = 0;
}

// ---------------------------------------------------------------------------
// Engine: the flush pipeline
//
// enqueue (caller, exclusive): swap out every queued program body and every
//   shard's queues into a Batch, hand it to the launcher.
// launcher thread: lay the batch out (every segment's place in the upload,
//   every solve's place in the result array), copy it into the pinned upload
//   buffer of its transfer set, then one H2D copy, the ingest, executor and
//   solve launches in phase order, the D2H of results and downloads, and a
//   fence.
// completer thread: wait for the fence, deliver downloads, run completions,
//   return released buffers to the depot and the bodies/queues for reuse.

namespace {

struct Phase
{
    enum Kind { EXEC, SOLVE } kind;
    size_t itemBegin, itemCount;    // exec items or solve items
    size_t solveBegin, solveCount;  // solve descs (SOLVE)
    uint32_t maxRows;               // largest m among them (SOLVE); largest OP_ROWS window (EXEC)
    size_t wideBegin = 0, wideCount = 0;   // k_ldpc items run before the exec launch (EXEC)
    int group = 0;                  // the programs' group (1: decoders, which the matrix jobs feed)
};

struct SegRef
{
    const ProgramBody::Segment* seg;
    uint32_t wordBase, words, itemBase;
    uint32_t tilesPerItem = 1;      // tiles one k_exec workgroup runs
    uint32_t wideBase = 0;          // first k_ldpc item of its wide rows
    uint64_t wideOff = 0;           // their scratch (bytes into the set's wideDev)
    uint32_t resultBase = 0;        // its body's first result word (gated batches)
};

} // namespace

struct Batch
{
    uint64_t ticket = 0;
    std::vector<ProgramBody*> bodies[2];   // by group
    std::vector<Shard::Queues> queues;     // detached shard queues
    std::vector<Shard*> queueOwner;
    unsigned set = 0;                      // transfer set (ticket % kSets)
    // layout (enqueue -> launcher)
    std::vector<Phase> phases;
    size_t upBytes = 0, nIngest = 0, nIngBlocks = 0;
    uint32_t maxIngest = 0;
    size_t oIngD = 0, oIngB = 0, oStream = 0, oItems = 0, oSD = 0, oSR = 0, oCoef = 0, oSI = 0, oWide = 0;
    size_t oGeD = 0, oGeIn = 0, nGe = 0;   // device matrix jobs: descs, inputs
    size_t geHead = 0;                      // bytes of the upload's head: the jobs and what they write
    bool allGated = false;                  // every solve of the submission is a chained job's
    uint32_t geMaxRows = 0, geMaxCols = 0;  // ... their largest matrix (k_ge's LDS)
    bool geChained = false;                 // a job writes into the upload (kGeChained)
    size_t oCopy = 0;                      // the download copy list (BeCopy records)
    uint64_t wideBase = 0;                 // this submission's k_ldpc scratch: bytes into the ring
    bool wideZero = false;                 // the ring wrapped: zero it before the first exec launch
    uint32_t resultWords = 0;
    std::vector<const Shard::Download*> dls;
    std::vector<BeCopy> copies;         // D2H ranges of launch_batch (scratch)
    uint8_t* upBase = nullptr;          // where the kernels read the upload: the set's device copy, or zero-copy
    EngineStats st;
    // launcher -> completer
    void* fence = nullptr;
    bool launched = false;
    std::vector<uint32_t> resultBase[2];
    struct Download
    {
        void* host;
        size_t off;
        uint32_t bytes;
    };
    std::vector<Download> downloads;
    std::vector<void*> marks;              // staged copies its device work waits for
    bool assembled = false;                // laid out (by enqueue, or by the launcher)
};

namespace {

// SGPU_TIMELINE=1: one stderr line per pipeline event (debugging aid)
const bool g_timeline = std::getenv("SGPU_TIMELINE") != nullptr;
void tl(const char* what, uint64_t ticket)
{
    if (g_timeline)
        std::fprintf(stderr, "eng %10.3f ms  %s t%llu\n", (double)now_ns() / 1e6, what,
                     (unsigned long long)ticket);
}

// the download area starts with the byte counters: the executor's expanded
// terms, then the solve's back-substitution source bytes and output bytes
constexpr size_t kAcctBytes = 32;

// below this many stream words a submission is assembled on the calling
// thread alone (the drop-in API's per-call flushes)
constexpr size_t kParallelWords = 1u << 16;
// flush assembly task sizes (bodies sealed, segments, ingest records and
// solves per pool task)
#ifndef SGPU_SEAL_CHUNK
#define SGPU_SEAL_CHUNK 32
#endif
#ifndef SGPU_SEG_CHUNK
#define SGPU_SEG_CHUNK 16
#endif
#ifndef SGPU_INGEST_CHUNK
#define SGPU_INGEST_CHUNK 8192
#endif
#ifndef SGPU_SOLVE_CHUNK
#define SGPU_SOLVE_CHUNK 64
#endif

// ---- compulsory bytes of an executor segment (Engine::set_measure_unique) --
std::atomic<bool> g_measureUnique{false};

struct Range
{
    uint64_t addr;
    uint32_t len;
};

// every distinct symbol counted once at the largest extent any op of the
// segment touches it with
uint64_t distinct_bytes(std::vector<Range>& v)
{
    std::sort(v.begin(), v.end(), [](const Range& a, const Range& b) { return a.addr < b.addr; });
    uint64_t total = 0;
    for (size_t i = 0; i < v.size();) {
        uint32_t len = v[i].len;
        size_t j = i + 1;
        for (; j < v.size() && v[j].addr == v[i].addr; ++j)
            len = std::max(len, v[j].len);
        total += len;
        i = j;
    }
    return total;
}

// The bytes one executor segment must move at the least: each source symbol
// read once (a window element or sum re-read by several rows of a batch is
// one read: the kernel stages them in LDS), each destination written once
// (and its kept prefix read once), the op stream itself read once.  The
// algorithmic bytes count every re-read; this does not.
uint64_t segment_unique_bytes(const ProgramBody::Segment& s, std::vector<Range>& rd, std::vector<Range>& wr)
{
    rd.clear();
    wr.clear();
    uint64_t words = 0;
    auto R = [&](uint64_t a, uint32_t n) {
        if (a && n)
            rd.push_back(Range{a, n});
    };
    auto W = [&](uint64_t a, uint32_t n, uint32_t valid) {
        if (a && n)
            wr.push_back(Range{a, n});
        R(a, std::min(valid, n));
    };
    for (const GfOp& op : s.ops) {
        words += op_words(op);
        const uint8_t* blk = s.rowsData.data() + (size_t)op.termBegin * 16;
        switch (op.kind) {
        case OP_LINCOMB:
            W(op.dst, op.n, op.valid);
            for (uint32_t t = 0; t < op.termCount; ++t)
                R(s.terms[op.termBegin + t].src, s.terms[op.termBegin + t].len);
            break;
        case OP_LITERAL:
            W(op.dst + op.n, op.valid, 0);
            break;
        case OP_ROWS: {
            const WinEntry* sums = reinterpret_cast<const WinEntry*>(blk);
            const WinEntry* win = sums + kRowSums;
            const SumUpdate* up = reinterpret_cast<const SumUpdate*>(win + op.valid);
            const RowItem* rows = reinterpret_cast<const RowItem*>(up + op.mix);
            for (unsigned k = 0; k < kRowSums; ++k)
                R(sums[k].src, sums[k].len);
            for (uint32_t e = (uint32_t)op.dst; e < op.valid; ++e)   // (from stageLo)
                R(win[e].src, win[e].len);
            for (uint32_t u = 0; u < op.mix; ++u)
                W((uint64_t)up[u].dstHi << 32 | up[u].dstLo, up[u].n, up[u].valid);
            for (uint32_t r = 0; r < op.n; ++r)
                W(rows[r].dst, rows[r].n + row_lit_len(rows[r].mask0), rows[r].valid);
            break;
        }
        case OP_COPIES: {
            const CopyItem* c = reinterpret_cast<const CopyItem*>(blk);
            for (uint32_t i = 0; i < op.n; ++i) {
                W(c[i].dst, c[i].len, 0);
                R(c[i].src, c[i].len);
            }
            break;
        }
        case OP_LINCOMBS: {
            const LcItem* it = reinterpret_cast<const LcItem*>(blk);
            for (uint32_t i = 0; i < op.n; ++i) {
                W(it[i].dst, std::max(it[i].n, it[i].litOffset + ((it[i].mixLit >> 8) & 0xff)), it[i].valid);
                const GfTerm* t = reinterpret_cast<const GfTerm*>(blk + (size_t)it[i].termStart * 16);
                for (uint32_t k = 0; k < it[i].termCount; ++k)
                    R(t[k].src, t[k].len);
            }
            break;
        }
        default:
            break;
        }
    }
    return words * 16 + distinct_bytes(rd) + distinct_bytes(wr);
}

} // namespace

void Engine::set_measure_unique(bool on) { g_measureUnique.store(on, std::memory_order_relaxed); }
bool Engine::measure_unique() { return g_measureUnique.load(std::memory_order_relaxed); }

void Engine::start_threads()
{
    stop_ = false;
    launcher_ = std::thread([this] {
        pthread_setname_np(pthread_self(), "sgpu-launch");
        launcher_loop();
    });
    completer_ = std::thread([this] {
        pthread_setname_np(pthread_self(), "sgpu-complete");
        completer_loop();
    });
}

void Engine::stop_threads()
{
    {
        std::lock_guard<std::mutex> g(qMu_);
        stop_ = true;
    }
    launchCv_.notify_all();
    completeCv_.notify_all();
    setCv_.notify_all();
    doneCv_.notify_all();
    if (launcher_.joinable())
        launcher_.join();
    if (completer_.joinable())
        completer_.join();
}

Batch* Engine::take_batch()
{
    std::vector<Shard*> shards;
    {
        std::lock_guard<std::mutex> g(shardsMu_);
        for (auto& s : shards_)
            shards.push_back(s.get());
    }
    Batch* b = nullptr;
    for (Shard* s : shards) {
        if (s->dirty.empty() && s->q.empty())
            continue;
        if (!b)
            b = new Batch;
        for (Program* p : s->dirty) {
            ProgramBody* body = p->b_;
            p->b_ = nullptr;
            p->shard_ = nullptr;
            if (body) {
                if (body->empty() && body->callbacks.empty())
                    ProgramBody::put(body);
                else
                    b->bodies[body->group].push_back(body);
            }
            if (p->group_ & 2)
                delete p;   // orphan of a freed instance (see ~Program)
        }
        s->dirty.clear();
        if (!s->q.empty()) {
            Shard::Queues next;
            {
                std::lock_guard<std::mutex> g(s->mu);
                if (!s->spare.empty()) {
                    next = std::move(s->spare.back());
                    s->spare.pop_back();
                }
            }
            b->queues.push_back(std::move(s->q));
            b->queueOwner.push_back(s);
            s->q = std::move(next);
        }
    }
    if (!b)
        return nullptr;
    const uint64_t ticket = ++nextTicket_;
    tl("enqueue", ticket);
    b->ticket = ticket;
    b->set = (unsigned)(ticket % kSets);
    {
        std::lock_guard<std::mutex> g(qMu_);
        b->marks.swap(pendingMarks_);
    }
    return b;
}


uint64_t Engine::enqueue()
{
    if (failed())
        return 0;
    std::lock_guard<std::mutex> sub(submitMu_);
    Batch* b = take_batch();
    if (!b)
        return nextTicket_;   // nothing queued: the latest submission covers everything
    const uint64_t ticket = b->ticket;
    // The batch is laid out by the launcher thread and its own pool, so the
    // caller goes back to driving instances at once (same-box A/B of the
    // headline, 5 interleaved runs each: median 6.34 vs 6.63 ms/step against
    // laying it out here, profiles/r4i_async_ab.txt).
    {
        std::lock_guard<std::mutex> g(qMu_);
        toLaunch_.push_back(b);   // (b belongs to the pipeline from here on)
        queuedSeen_.fetch_add(1, std::memory_order_release);
    }
    launchCv_.notify_one();
    setCv_.notify_all();   // (a launcher waiting for a set to take requests re-checks toLaunch_)
    return ticket;
}


bool Engine::wait(uint64_t ticket)
{
    std::unique_lock<std::mutex> lk(qMu_);
    doneCv_.wait(lk, [&] { return stop_ || doneTicket_ >= ticket; });
    return !failed();
}

bool Engine::flush_and_sync(InstanceLock* detach)
{
    if (failed())
        return false;
    std::unique_lock<std::mutex> sub(submitMu_);
    if (detach)
        return flush_requested(sub, *detach);
    Batch* b;
    uint64_t last;
    b = take_batch();
    last = nextTicket_;
    if (!b) {
        // (an earlier submission took this caller's work: wait for it)
        sub.unlock();
        return wait(last) && last != 0;
    }
    const uint64_t ticket = b->ticket;
    bool inl = false;
    // (with nothing queued or running the caller lays out and launches its
    // own submission, and the launcher takes nothing while inlineBusy_ is
    // set; the hand-off costs a per-call flush ~15 us,
    // profiles/r4ao_dropin_ab.txt)
    {
        std::lock_guard<std::mutex> g(qMu_);
        // Inline only when the ticket's transfer set is free right now, and
        // claimed in this same critical section: a later ticket of the same
        // set (T + kSets) could otherwise claim it first and then wait in
        // toLaunch_ behind inlineBusy_ while this caller waits for the set.
        if (toLaunch_.empty() && toComplete_.empty() && !launching_ && !completing_ && !inlineBusy_ &&
            flushReq_ == takenReq_ && doneTicket_ + 1 == ticket && sets_[b->set].busyTicket == 0) {
            sets_[b->set].busyTicket = ticket;
            inlineBusy_ = true;   // (the launcher waits: its stream order stays ticket order)
            inl = true;
        }
    }
    if (!inl) {
        {
            std::lock_guard<std::mutex> g(qMu_);
            toLaunch_.push_back(b);
            queuedSeen_.fetch_add(1, std::memory_order_release);
        }
        sub.unlock();
        launchCv_.notify_one();
        setCv_.notify_all();   // (a launcher waiting for a set to take requests re-checks toLaunch_)
        return wait(ticket) && !failed();
    }
    return run_inline(b, sub);
}

bool Engine::flush_requested(std::unique_lock<std::mutex>& sub, InstanceLock& detach)
{
    // The drop-in API's flush.  An idle pipeline: the caller detaches, lays
    // out and launches the submission itself (one stream's per-call
    // latency).  Otherwise the caller files a request and the launcher
    // detaches the queued work once the next ticket's transfer set is free,
    // so every call the other application threads queued meanwhile rides in
    // the same submission: concurrent callers share few large submissions
    // instead of paying one submission each behind the transfer sets.
    bool idle;
    {
        std::lock_guard<std::mutex> g(qMu_);
        const uint64_t next = nextTicket_.load(std::memory_order_relaxed) + 1;
        idle = toLaunch_.empty() && toComplete_.empty() && !launching_ && !completing_ && !inlineBusy_ &&
               flushReq_ == takenReq_ && doneTicket_ + 1 == next && sets_[next % kSets].busyTicket == 0;
        if (idle)
            inlineBusy_ = true;   // (the launcher takes nothing until this caller has launched)
    }
    if (!idle) {
        sub.unlock();
        uint64_t my;
        {
            std::lock_guard<std::mutex> g(qMu_);
            my = ++flushReq_;
        }
        launchCv_.notify_one();
        std::unique_lock<std::mutex> lk(qMu_);
        doneCv_.wait(lk, [&] { return stop_ || takenReq_ >= my; });
        const uint64_t t = reqTicket_;   // (covers this caller's work: every ticket up to it)
        doneCv_.wait(lk, [&] { return stop_ || doneTicket_ >= t; });
        return t != 0 && doneTicket_ >= t && !failed();
    }
    Batch* b;
    {
        std::unique_lock<InstanceLock> w(detach);
        b = take_batch();
    }
    if (!b) {
        // (an earlier submission took this caller's work: wait for it)
        const uint64_t last = nextTicket_;
        {
            std::lock_guard<std::mutex> g(qMu_);
            inlineBusy_ = false;
        }
        sub.unlock();
        launchCv_.notify_one();
        return wait(last) && last != 0;
    }
    {
        std::lock_guard<std::mutex> g(qMu_);
        sets_[b->set].busyTicket = b->ticket;   // (free: checked above, and nobody took a ticket since)
    }
    return run_inline(b, sub);
}

bool Engine::run_inline(Batch* b, std::unique_lock<std::mutex>& sub)
{
    tl("inline", b->ticket);
    assemble_batch(*b, pool());   // (the set was claimed by the caller)
    if (!failed())
        launch_batch(*b);
    {
        // Launched: later tickets follow it on the stream, so the launcher
        // may lay out and launch other threads' submissions while this caller
        // waits for its fence; the completer publishes them only after this
        // ticket.
        std::lock_guard<std::mutex> g(qMu_);
        inlineBusy_ = false;
    }
    sub.unlock();   // (the next submission may be laid out while this one runs)
    launchCv_.notify_one();
    if (complete_batch(*b))
        reclaim_batch(*b);
    {
        std::lock_guard<std::mutex> g(qMu_);
        if (sets_[b->set].busyTicket == b->ticket)
            sets_[b->set].busyTicket = 0;
        doneTicket_ = b->ticket;
        doneSeen_.store(b->ticket, std::memory_order_release);
    }
    setCv_.notify_all();
    doneCv_.notify_all();
    delete b;
    return !failed();
}

Batch* Engine::take_requested()
{
    // Wait for the next ticket's transfer set before detaching: calls that
    // arrive meanwhile join this submission.
    for (;;) {
        uint64_t next;
        {
            std::unique_lock<std::mutex> lk(qMu_);
            next = nextTicket_.load(std::memory_order_acquire) + 1;
            setCv_.wait(lk, [&] { return stop_ || !toLaunch_.empty() || sets_[next % kSets].busyTicket == 0; });
            if (stop_ || !toLaunch_.empty())
                return nullptr;   // (queued submissions go first)
        }
        std::lock_guard<std::mutex> sub(submitMu_);
        if (nextTicket_.load(std::memory_order_relaxed) + 1 != next)
            continue;   // (a ticket was handed out meanwhile)
        uint64_t reqs;
        {
            std::lock_guard<std::mutex> g(qMu_);
            reqs = flushReq_;
        }
        Batch* b;
        {
            std::unique_lock<InstanceLock> w(instMu_);
            b = take_batch();
        }
        {
            std::lock_guard<std::mutex> g(qMu_);
            takenReq_ = reqs;
            reqTicket_ = nextTicket_.load(std::memory_order_relaxed);
        }
        doneCv_.notify_all();
        return b;
    }
}

bool Engine::flush()
{
    uint64_t prev;
    {
        std::lock_guard<std::mutex> sub(submitMu_);
        prev = nextTicket_;
    }
    enqueue();
    // complete what was in flight before this submission (one flush in flight)
    return wait(prev) && !failed();
}

void Engine::launcher_loop()
{
    uint64_t taken = 0;   // batches taken from toLaunch_
    for (;;) {
        Batch* b = nullptr;
        {
            std::unique_lock<std::mutex> lk(qMu_);
            launchCv_.wait(lk, [&] {
                return stop_ || (!inlineBusy_ && (!toLaunch_.empty() || flushReq_ > takenReq_));
            });
            if (stop_)
                return;
            if (!toLaunch_.empty()) {
                b = toLaunch_.front();
                toLaunch_.pop_front();
                ++taken;
            }
            launching_ = true;
        }
        if (!b) {
            // drop-in flush requests: detach everything queued so far
            b = take_requested();
            if (!b) {
                std::lock_guard<std::mutex> g(qMu_);
                launching_ = false;
                continue;
            }
        }
        if (!b->assembled && !failed()) {
            claim_set(*b);
            assemble_batch(*b, asm_pool());
            tl("assembled", b->ticket);
        }
        tl("launch begin", b->ticket);
        if (!failed())
            launch_batch(*b);
        tl("launch end", b->ticket);
        {
            std::lock_guard<std::mutex> g(qMu_);
            toComplete_.push_back(b);
            launching_ = false;
        }
        completeCv_.notify_one();
    }
}

// Lay the batch out and copy it into its pinned upload buffer (caller's
// thread, in parallel on the worker pool for large batches):
//   1. every open Siamese row batch is sealed (parallel over bodies);
//   2. a sequential pass fixes every segment's place in the upload and its
//      work items, and every solve's place in the result array;
//   3. segments, solve data and ingest descriptors are copied (parallel).
void Engine::claim_set(Batch& b)
{
    // this ticket's transfer set must be free (its previous user done)
    std::unique_lock<std::mutex> lk(qMu_);
    setCv_.wait(lk, [&] { return stop_ || sets_[b.set].busyTicket == 0; });
    sets_[b.set].busyTicket = b.ticket;
}

WorkerPool& Engine::asm_pool()
{
    // the launcher's own pool: the application may be running a fork-join
    // on pool() while a batch is laid out (SIAMESE_AMD_ASM_THREADS, default 4)
    if (!asmPool_) {
        // (4 measured best on the box's 16-core share: 6.07/5.93/6.34 ms
        // per step vs 7.88/6.34/6.98 with 8, profiles/r4p_threads_ab.txt)
        const char* v = std::getenv("SIAMESE_AMD_ASM_THREADS");
        const int n = v ? std::atoi(v) : 4;
        asmPool_.reset(new WorkerPool((unsigned)std::max(1, std::min(64, n)), 0, "sgpu-assemble"));
    }
    return *asmPool_;
}

void Engine::assemble_batch(Batch& bt, WorkerPool& wp)
{
    bt.assembled = true;
    const uint64_t t0 = now_ns();
    XferSet& xs = sets_[bt.set];
    EngineStats& st = bt.st;
    size_t totalBodies = bt.bodies[0].size() + bt.bodies[1].size();
    size_t approxWords = 0;
    for (const Shard::Queues& q : bt.queues)
        approxWords += q.ingest.size() * 2;
    for (int g = 0; g < 2; ++g)
        for (ProgramBody* p : bt.bodies[g])
            for (size_t k = 0; k < p->nsegs; ++k)
                approxWords += p->segs[k].ops.size() * 2 + p->segs[k].terms.size() +
                               p->segs[k].rowsWords + p->rb.win.size() + p->rb.rows.size() * 3;
    const bool parallel = approxWords >= kParallelWords;
    auto run = [&](size_t n, const std::function<void(size_t)>& fn) {
        if (parallel)
            wp.run(n, fn);
        else
            for (size_t i = 0; i < n; ++i)
                fn(i);
    };

    // ---- 1. seal -------------------------------------------------------------
    // (task sizes: small enough that a fork-join's tail stays short)
    constexpr size_t kSealChunk = SGPU_SEAL_CHUNK;
    run((totalBodies + kSealChunk - 1) / kSealChunk, [&](size_t c) {
        for (size_t i = c * kSealChunk; i < std::min(totalBodies, c * kSealChunk + kSealChunk); ++i) {
            const size_t n0 = bt.bodies[0].size();
            (i < n0 ? bt.bodies[0][i] : bt.bodies[1][i - n0])->rows_close();
        }
    });

    // ---- 2. layout -----------------------------------------------------------
    uint32_t resultWords = 0;
    for (int g = 0; g < 2; ++g)
        for (ProgramBody* p : bt.bodies[g]) {
            bt.resultBase[g].push_back(resultWords);
            resultWords += p->resultWords;
        }
    bt.resultWords = resultWords;

    std::vector<SegRef> segs;
    std::vector<Phase>& phases = bt.phases;
    std::vector<SolveDesc> sdescs;
    struct SolveRef
    {
        const ProgramBody::PendingSolve* ps;
        size_t rowBase, coefBase;
    };
    std::vector<SolveRef> srefs;
    size_t nSolveRows = 0, nCoef = 0;
    std::vector<SolveItem> sitems;
    size_t nOps = 0, nTerms = 0, nWords = 0, nItems = 0, nWide = 0;
    uint64_t wideBytes = 0, tBytes = 0;
    for (int g = 0; g < 2; ++g) {
        size_t maxSegs = 0;
        for (ProgramBody* p : bt.bodies[g])
            maxSegs = std::max(maxSegs, p->nsegs);
        for (size_t k = 0; k < maxSegs; ++k) {
            Phase ex{Phase::EXEC, nItems, 0, 0, 0, kNoRows};
            const size_t segBegin = segs.size();
            for (size_t pi = 0; pi < bt.bodies[g].size(); ++pi) {
                const ProgramBody* p = bt.bodies[g][pi];
                if (k >= p->nsegs)
                    continue;
                const ProgramBody::Segment& s = p->segs[k];
                if (s.ops.empty())
                    continue;
                for (const GfOp& op : s.ops)
                    if (op.kind == OP_ROWS)
                        ex.maxRows = ex.maxRows == kNoRows ? op.valid : std::max(ex.maxRows, op.valid);
                const size_t words = kOpWords * s.ops.size() + s.terms.size() + s.rowsWords;
                segs.push_back(SegRef{&s, (uint32_t)nWords, (uint32_t)words, 0});
                segs.back().resultBase = bt.resultBase[g][pi];
                nOps += s.ops.size();
                nTerms += s.terms.size();
                nWords += words;
            }
#if SGPU_EXEC_LPT
            // Longest op lists first: workgroups are dispatched in blockIdx
            // order and a launch runs in a few rounds of workgroups per CU,
            // so the short segments fill the last round's tail.
            std::stable_sort(segs.begin() + (long)segBegin, segs.end(),
                             [](const SegRef& a, const SegRef& b) { return a.words > b.words; });
#endif
            {
                // Runs of a segment's tiles per workgroup once the launch has
                // more work than the chip runs at once: a workgroup then
                // loads each OP_ROWS table and draws its row plans once for
                // all of its tiles (a single stream's few tiles stay spread
                // over as many workgroups).
                // Runs only for segments with row batches (their tables and
                // plans are what a run shares), of tpi tiles when the launch
                // has more tiles than workgroup slots; a segment much heavier
                // than the launch's average (op-stream words as the per-tile
                // work: a C2 decode beside one-row encodes) gets a shorter
                // run, or it becomes the launch's tail (C2 k_exec 4.25 vs
                // 10.7 ms per run with uniform runs, tools/leg_ab.sh)
                size_t phaseTiles = 0;
                double words = 0;
                for (size_t i = segBegin; i < segs.size(); ++i) {
                    const size_t t = (segs[i].seg->maxExtent + kExecTileBytes - 1) / kExecTileBytes;
                    phaseTiles += t;
                    words += (double)t * segs[i].words;
                }
                const double avg = phaseTiles ? words / (double)phaseTiles : 0.0;   // words per tile
                const size_t tpi = std::min<size_t>(
                    kExecRunMax, std::max<size_t>(1, (phaseTiles + SGPU_EXEC_GROUPS - 1) / SGPU_EXEC_GROUPS));
                uint32_t ib = (uint32_t)ex.itemBegin;
                for (size_t i = segBegin; i < segs.size(); ++i) {
                    const size_t tiles = (segs[i].seg->maxExtent + kExecTileBytes - 1) / kExecTileBytes;
                    size_t run = 1;
                    if (segs[i].seg->rowsWords && tpi > 1) {
                        const double heavy = segs[i].words / (2.0 * avg);
                        run = heavy > 1.0 ? std::max<size_t>(1, (size_t)((double)tpi / heavy)) : tpi;
                    }
                    segs[i].itemBase = ib;
                    segs[i].tilesPerItem = (uint32_t)run;
                    ib += (uint32_t)((tiles + run - 1) / run);
                }
                nItems = ib;
            }
            ex.itemCount = nItems - ex.itemBegin;
            ex.wideBegin = nWide;
            for (size_t i = segBegin; i < segs.size(); ++i) {
                const ProgramBody::Segment& s = *segs[i].seg;
                if (s.wide.empty())
                    continue;
                segs[i].wideBase = (uint32_t)nWide;
                segs[i].wideOff = wideBytes;
                nWide += s.wideItems;
                wideBytes += s.wideBytes;
            }
            ex.wideCount = nWide - ex.wideBegin;
            ex.group = g;
            if (ex.itemCount)
                phases.push_back(ex);

            Phase sv{Phase::SOLVE, sitems.size(), 0, sdescs.size(), 0, 0};
            for (size_t pi = 0; pi < bt.bodies[g].size(); ++pi) {
                const ProgramBody* p = bt.bodies[g][pi];
                if (k >= p->nsolves)
                    continue;
                const ProgramBody::PendingSolve& ps = p->solves[k];
                SolveDesc d = ps.desc;
                d.result += bt.resultBase[g][pi];
                if (d.gate)
                    d.gate += bt.resultBase[g][pi];
                d.rowBegin = (uint32_t)nSolveRows;
                d.coefOffset = nCoef;
                ps.asmRow = (uint32_t)nSolveRows;
                ps.asmCoef = (uint32_t)nCoef;
                srefs.push_back(SolveRef{&ps, nSolveRows, nCoef});
                nSolveRows += ps.rows.size();
                nCoef += ps.coef.size();
                const uint32_t sidx = (uint32_t)sdescs.size();
                sdescs.push_back(d);
                sv.maxRows = std::max(sv.maxRows, d.m);
                // (tile 0 always runs: it publishes the solve's result words)
                const uint32_t tb = solve_tile_bytes(d.m);
                uint32_t t = 0;
                do
                    sitems.push_back(SolveItem{sidx, t});
                while ((t += tb) < d.maxBytes);
            }
#if SGPU_EXEC_LPT
            // largest solves first (the serial pivot chain grows with m)
            std::stable_sort(sitems.begin() + (long)sv.itemBegin, sitems.end(),
                             [&](const SolveItem& a, const SolveItem& b) {
                                 return sdescs[a.solve].m > sdescs[b.solve].m;
                             });
#endif
            sv.itemCount = sitems.size() - sv.itemBegin;
            sv.solveCount = sdescs.size() - sv.solveBegin;
            if (solve_split((uint32_t)sv.solveCount, sv.maxRows))
                for (size_t i = sv.solveBegin; i < sdescs.size(); ++i) {
                    // the inverse's scratch (matrix-core path), in the k_ldpc ring
                    // after this submission's k_ldpc scratch (1 + its offset
                    // there until placed below)
                    const uint32_t tb = solve_t_bytes(sdescs[i].m);
                    if (tb) {
                        sdescs[i].tinv = 1 + tBytes;
                        tBytes += tb;
                        sdescs[i].xout = 1 + tBytes;
                        tBytes += (solve_x_bytes(sdescs[i].m, sdescs[i].maxBytes) + 255u) & ~(uint64_t)255u;
                    }
                }
            sv.group = g;
            if (sv.solveCount)
                phases.push_back(sv);
        }
    }

    // device matrix jobs (any body, either group: they read only their input)
    struct GeRef
    {
        const ProgramBody::PendingGe* g;
        size_t inOff;
    };
    std::vector<GeDesc> gdescs;
    std::vector<GeRef> grefs;
    size_t geInBytes = 0;
    for (int g = 0; g < 2; ++g)
        for (size_t pi = 0; pi < bt.bodies[g].size(); ++pi) {
            const ProgramBody* p = bt.bodies[g][pi];
            for (size_t k = 0; k < p->nges; ++k) {
                const ProgramBody::PendingGe& ge = p->ges[k];
                GeDesc d;
                std::memset(&d, 0, sizeof(d));
                d.in = (uint32_t)geInBytes;
                d.result = ge.result + bt.resultBase[g][pi];
                d.rows = ge.rows;
                d.cols = ge.cols;
                d.pickLen = ge.pickLen;
                if (ge.chained && ge.solve < p->nsolves) {
                    d.flags = kGeChained;
                    d.solveRow = p->solves[ge.solve].asmRow;
                    d.solveCoef = p->solves[ge.solve].asmCoef;
                    bt.geChained = true;
                }
                bt.geMaxRows = std::max<uint32_t>(bt.geMaxRows, ge.rows);
                bt.geMaxCols = std::max<uint32_t>(bt.geMaxCols, ge.cols);
                gdescs.push_back(d);
                grefs.push_back(GeRef{&ge, geInBytes});
                geInBytes = align16(geInBytes + ge.in.size());
            }
        }
    bt.nGe = gdescs.size();

    constexpr size_t kIngestChunk = SGPU_INGEST_CHUNK;
    size_t nIngest = 0, stageBytes = 0, nIngBlocks = 0;
    std::vector<size_t> descBase, stageBase;
    // the k_ingest block table's first entry of every ingest chunk (a run of
    // n symbols takes ceil(n / kIngestWaves) entries)
    std::vector<std::vector<size_t>> blockBase(bt.queues.size());
    for (size_t qi = 0; qi < bt.queues.size(); ++qi) {
        const Shard::Queues& q = bt.queues[qi];
        descBase.push_back(nIngest);
        stageBase.push_back(stageBytes);
        nIngest += q.ingest.size();
        bt.maxIngest = std::max(bt.maxIngest, q.maxIngest);
        stageBytes = align16(stageBytes + q.hostStage.size());
        for (size_t i = 0; i < q.ingest.size(); ++i) {
            if (i % kIngestChunk == 0)
                blockBase[qi].push_back(nIngBlocks);
            const uint32_t n = q.ingest[i].d.count ? q.ingest[i].d.count : 1u;
            nIngBlocks += (n + kIngestWaves - 1) / kIngestWaves;
        }
    }
    bt.nIngest = nIngest;
    bt.nIngBlocks = nIngBlocks;

    // The matrix jobs, then the solves' rows and coefficients (which a chained
    // job rewrites), at the head of the upload: that head is copied first and
    // k_ge starts on it while the rest is still crossing the bus
    // (launch_batch).
    size_t off = 0;
    bt.oGeD = off;
    off = align16(off + gdescs.size() * sizeof(GeDesc));
    bt.oGeIn = off;
    off = align16(off + geInBytes);
    bt.oSR = off;
    off = align16(off + nSolveRows * sizeof(SolveRow));
    bt.oCoef = off;
    off = align16(off + nCoef);
    bt.geHead = off;
    bt.allGated = !sdescs.empty();
    for (const SolveDesc& d : sdescs)
        bt.allGated = bt.allGated && d.gate != 0;
    const size_t oStage = off;
    off = align16(off + stageBytes);
    bt.oIngD = off;
    off = align16(off + nIngest * sizeof(IngestDesc));
    bt.oIngB = off;
    off = align16(off + nIngBlocks * sizeof(uint32_t));
    bt.oStream = off;
    off = align16(off + nWords * 16);
    bt.oItems = off;
    off = align16(off + nItems * sizeof(ExecItem));
    bt.oSD = off;
    off = align16(off + sdescs.size() * sizeof(SolveDesc));
    bt.oSI = off;
    off = align16(off + sitems.size() * sizeof(SolveItem));
    bt.oWide = off;
    off = align16(off + nWide * sizeof(LdpcItem));
    // the download copy list (the counters and results, then every range)
    size_t nDownloads = 0;
    for (const Shard::Queues& q : bt.queues)
        nDownloads += q.downloads.size();
    bt.oCopy = off;
    off = align16(off + (nDownloads + 1) * sizeof(BeCopy));
    bt.upBytes = off;
    if (bt.upBytes)
        ensure_up(xs, bt.upBytes);
    // A small upload is not copied: the kernels read it from the pinned
    // buffer over the bus (zero-copy), which skips a copy and its hand-off
    // on the latency-bound paths (SIAMESE_AMD_ZEROCOPY_UP bytes at most,
    // default 32 KiB; 0 disables).
    constexpr size_t kZeroCopyUp = 32768;
    // (a chained matrix job writes its solve's rows and coefficients into
    // the upload: the device copy then)
    bt.upBase = (xs.upHostDev && bt.upBytes <= kZeroCopyUp && !bt.geChained) ? xs.upHostDev : xs.upDev;
    if (wideBytes) {
        // k_ldpc scratch comes from the set's ring, which is zeroed as a whole
        // when it wraps (not per submission: most flushes then need no memset)
        const uint64_t need = wideBytes;
        if (xs.wideUsed + need > xs.wideCap) {
            ensure_wide(xs, std::max<size_t>(need, 16u << 20));
            xs.wideUsed = 0;
            bt.wideZero = true;
        }
        bt.wideBase = xs.wideUsed;
        xs.wideUsed += need;
    }
    if (tBytes) {
        // the solves' inverses and results: their own scratch, from its start
        // (sharing the ring made the headline zero 16 MiB every submission or
        // two, 134 MB of the step's traffic, profiles/r6_traffic.json of r6e)
        ensure_solve(xs, tBytes);
        const uint64_t tBase = (uint64_t)(uintptr_t)xs.solveDev;
        for (SolveDesc& d : sdescs)
            if (d.tinv) {
                d.tinv = tBase + (d.tinv - 1);
                d.xout = tBase + (d.xout - 1);
            }
    }

    // ---- 3. copy into the pinned upload buffer -------------------------------
    uint8_t* up = xs.upHost;
    const uint64_t stageDev = (uint64_t)(uintptr_t)(bt.upBase + oStage);
    constexpr size_t kSegChunk = SGPU_SEG_CHUNK;
    constexpr size_t kSolveChunk = SGPU_SOLVE_CHUNK;
    struct Task
    {
        int kind;   // 0 = segments, 1 = ingest chunk, 2 = solves, 3 = matrix jobs
        size_t a, b;
    };
    std::vector<Task> tasks;
    for (size_t i = 0; i < segs.size(); i += kSegChunk)
        tasks.push_back(Task{0, i, std::min(segs.size(), i + kSegChunk)});
    for (size_t i = 0; i < grefs.size(); i += kSolveChunk)
        tasks.push_back(Task{3, i, std::min(grefs.size(), i + kSolveChunk)});
    for (size_t i = 0; i < srefs.size(); i += kSolveChunk)
        tasks.push_back(Task{2, i, std::min(srefs.size(), i + kSolveChunk)});
    for (size_t qi = 0; qi < bt.queues.size(); ++qi)
        for (size_t c = 0; c < std::max<size_t>(1, bt.queues[qi].ingest.size()); c += kIngestChunk)
            tasks.push_back(Task{1, qi, c});
    const bool measureUnique = measure_unique();
    std::atomic<uint64_t> uniqueBytes{0};
    run(tasks.size(), [&](size_t ti) {
        const Task& t = tasks[ti];
        if (t.kind == 0) {
            if (measureUnique) {
                std::vector<Range> rd, wr;
                uint64_t u = 0;
                for (size_t si = t.a; si < t.b; ++si)
                    u += segment_unique_bytes(*segs[si].seg, rd, wr);
                uniqueBytes.fetch_add(u, std::memory_order_relaxed);
            }
            for (size_t si = t.a; si < t.b; ++si) {
                const SegRef& r = segs[si];
                const ProgramBody::Segment& s = *r.seg;
                uint8_t* w = up + bt.oStream + (size_t)r.wordBase * 16;
                size_t wi = 0;                                      // next wide row
                LdpcItem* wItem = (LdpcItem*)(up + bt.oWide) + r.wideBase;
                uint64_t wOff = bt.wideBase + r.wideOff;
                size_t gi = 0;   // next gated range
                for (uint32_t oi = 0; oi < (uint32_t)s.ops.size(); ++oi) {
                    const GfOp& op = s.ops[oi];
                    std::memcpy(w, &op, sizeof(GfOp));
                    if (op.kind != OP_LITERAL) {
                        // termBegin on the device: the op's gate, 1 + a result
                        // word (ops.h GeDesc), or 0
                        while (gi < s.gates.size() && s.gates[gi].opEnd <= oi)
                            ++gi;
                        const bool gated = gi < s.gates.size() && s.gates[gi].opBegin <= oi;
                        reinterpret_cast<GfOp*>(w)->termBegin = gated ? 1u + s.gates[gi].word + r.resultBase : 0u;
                    }
                    w += sizeof(GfOp);
                    if (op.kind == OP_ROWS || op.kind == OP_COPIES || op.kind == OP_LINCOMBS) {
                        const size_t bytes = (size_t)op.termCount * 16;   // block (rows_close)
                        std::memcpy(w, s.rowsData.data() + (size_t)op.termBegin * 16, bytes);
                        // wide rows of this batch: their scratch pair as the
                        // appended window entries, and their k_ldpc items
                        const uint64_t winDev = (uint64_t)(uintptr_t)(bt.upBase + (w - up)) + kRowSums * 16;
                        for (; wi < s.wide.size() && s.wide[wi].op == oi; ++wi) {
                            const ProgramBody::Segment::Wide& x = s.wide[wi];
                            const uint32_t span = (x.n + kLdpcTileBytes - 1) / kLdpcTileBytes * kLdpcTileBytes;
                            const uint64_t dst = (uint64_t)(uintptr_t)xs.wideDev + wOff;
                            wOff += 2 * (uint64_t)span;
                            WinEntry* e = reinterpret_cast<WinEntry*>(w + (size_t)(kRowSums + x.entry) * 16);
                            e[0].src = dst;
                            e[0].len = x.n;
                            e[1].src = dst + span;
                            e[1].len = x.n;
                            const uint32_t pairs = (x.N + kPairRate - 1) / kPairRate;
                            const uint32_t ppi = ldpc_pairs_per_item(x.n);
                            for (uint32_t t = 0; t < x.n; t += kLdpcTileBytes)
                                for (uint32_t p0 = 0; p0 < pairs; p0 += ppi) {
                                    LdpcItem& it = *wItem++;
                                    it.win = winDev;
                                    it.dst = dst;
                                    it.span = span;
                                    it.n = x.n;
                                    it.row = x.row;
                                    it.N = x.N;
                                    it.off = x.off;
                                    it.tileBase = t;
                                    it.pair0 = p0;
                                    it.pair1 = std::min(pairs, p0 + ppi);
                                }
                        }
                        w += bytes;
                    } else if (op.kind == OP_LINCOMB && op.termCount) {
                        const size_t bytes = (size_t)op.termCount * sizeof(GfTerm);
                        std::memcpy(w, s.terms.data() + op.termBegin, bytes);
                        w += bytes;
                    }
                }
                ExecItem* items = (ExecItem*)(up + bt.oItems) + r.itemBase;
                const uint32_t nOpsSeg = (uint32_t)s.ops.size();
                const uint32_t tiles = (s.maxExtent + kExecTileBytes - 1) / kExecTileBytes;
                uint32_t n = 0;
                for (uint32_t t = 0; t < tiles; t += r.tilesPerItem)
                    items[n++] = ExecItem{r.wordBase, r.words, nOpsSeg,
                                          exec_tiles(t, std::min(r.tilesPerItem, tiles - t))};
            }
        } else if (t.kind == 3) {
            for (size_t i = t.a; i < t.b; ++i)
                std::memcpy(up + bt.oGeIn + grefs[i].inOff, grefs[i].g->in.data(), grefs[i].g->in.size());
        } else if (t.kind == 2) {
            for (size_t i = t.a; i < t.b; ++i) {
                const SolveRef& r = srefs[i];
                std::memcpy(up + bt.oSR + r.rowBase * sizeof(SolveRow), r.ps->rows.data(),
                            r.ps->rows.size() * sizeof(SolveRow));
                std::memcpy(up + bt.oCoef + r.coefBase, r.ps->coef.data(), r.ps->coef.size());
            }
        } else {
            const Shard::Queues& q = bt.queues[t.a];
            IngestDesc* descs = (IngestDesc*)(up + bt.oIngD) + descBase[t.a];
            const size_t end = std::min(q.ingest.size(), t.b + kIngestChunk);
            uint32_t* blk = t.b < q.ingest.size() ? (uint32_t*)(up + bt.oIngB) + blockBase[t.a][t.b / kIngestChunk]
                                                  : nullptr;
            for (size_t i = t.b; i < end; ++i) {
                IngestDesc d = q.ingest[i].d;
                if (q.ingest[i].hostOffset >= 0)
                    d.src = stageDev + stageBase[t.a] + (uint64_t)q.ingest[i].hostOffset;
                descs[i] = d;
                const uint32_t di = (uint32_t)(descBase[t.a] + i);
                const uint32_t n = d.count ? d.count : 1u;
                for (uint32_t g = 0; g * kIngestWaves < n; ++g)
                    *blk++ = di << 4 | g;
            }
            if (t.b == 0 && !q.hostStage.empty())
                std::memcpy(up + oStage + stageBase[t.a], q.hostStage.data(), q.hostStage.size());
        }
    });
    if (!sdescs.empty()) {
        std::memcpy(up + bt.oSD, sdescs.data(), sdescs.size() * sizeof(SolveDesc));
        std::memcpy(up + bt.oSI, sitems.data(), sitems.size() * sizeof(SolveItem));
    }
    if (!gdescs.empty())
        std::memcpy(up + bt.oGeD, gdescs.data(), gdescs.size() * sizeof(GeDesc));

    // download area: the byte counters (kAcctBytes), the solve results, then
    // each requested range
    size_t dOff = align16(kAcctBytes + (size_t)resultWords * 4);
    for (const Shard::Queues& q : bt.queues)
        for (const Shard::Download& d : q.downloads) {
            bt.downloads.push_back(Batch::Download{d.host, dOff, d.bytes});
            bt.dls.push_back(&d);
            dOff = align16(dOff + d.bytes);
        }
    ensure_down(xs, dOff);
    {
        // the same list for the device (one copy kernel however many ranges,
        // launch_batch): host sides as the device addresses them
        std::vector<BeCopy>& cp = bt.copies;
        cp.clear();
        cp.push_back(BeCopy{(uint64_t)(uintptr_t)xs.downHost, (uint64_t)(uintptr_t)xs.downDev,
                            kAcctBytes + (uint64_t)resultWords * 4});
        for (size_t i = 0; i < bt.dls.size(); ++i)
            cp.push_back(BeCopy{(uint64_t)(uintptr_t)(xs.downHost + bt.downloads[i].off), bt.dls[i]->dev,
                                bt.dls[i]->bytes});
        if (xs.downHostDev) {
            BeCopy* dl = (BeCopy*)(up + bt.oCopy);
            const uint64_t shift = (uint64_t)(uintptr_t)xs.downHostDev - (uint64_t)(uintptr_t)xs.downHost;
            for (size_t i = 0; i < cp.size(); ++i)
                dl[i] = BeCopy{cp[i].dst + shift, cp[i].src, cp[i].bytes};
        }
    }

    st.flushes = 1;
    st.launches = phases.size() + (nIngest ? 1 : 0) + (gdescs.empty() ? 0 : 1);
    st.ops = nOps;
    st.terms = nTerms;
    st.solves = sdescs.size();
    st.ingests = nIngest;
    st.uploadBytes = bt.upBytes;
    st.execUniqueBytes = uniqueBytes.load(std::memory_order_relaxed);
    st.assembleNs = now_ns() - t0;
}

// The matrix jobs in order on the codec stream, the rest of the upload and
// k_ingest beside them (launch_batch).  Traces of both arrangements
// (tools/r6_trace_libs.sh): a round's first k_exec starts 150 us after its
// first copy against 157 with the jobs on the side stream; a cross-stream
// wait costs 16-23 us before the next kernel even when satisfied, and a
// kernel starts 12-20 us after a copy on its queue.  Headline within noise
// (profiles/r6l_ge_codec_stream_ab.txt).
constexpr bool kGeOnCodecStream = true;

void Engine::launch_batch(Batch& bt)
{
    XferSet& xs = sets_[bt.set];
    EngineStats& st = bt.st;

    // originals the application staged on the transfer stream (stage_in)
    for (void* m : bt.marks) {
        be_wait_mark(m);
        be_mark_release(m);
    }
    bt.marks.clear();
    // The upload.  With matrix jobs its head (the jobs' inputs and the solve
    // rows and coefficients they rewrite) is copied first and the jobs run on
    // it in order on the codec stream, while the rest of the upload and
    // k_ingest run beside them on the side stream, joined before the first
    // phase.  (The other way round -- the jobs on the side stream -- the
    // codec stream's join waited on a job that ended about when k_ingest did,
    // and a cross-stream wait that is not yet satisfied costs ~24 us of
    // latency on the join; a satisfied one costs next to nothing.)
    const bool copyUp = bt.upBytes && bt.upBase == xs.upDev;
    const size_t head = (copyUp && bt.nGe) ? bt.geHead : 0;
    uint64_t* acctDev = (uint64_t*)xs.downDev;
    uint32_t* resultsDev = (uint32_t*)(xs.downDev + kAcctBytes);
    const BeCopy rest{(uint64_t)(uintptr_t)xs.upDev + head, (uint64_t)(uintptr_t)xs.upHost + head,
                      bt.upBytes - head};
    bool ingested = false;
    if (bt.nGe && head && kGeOnCodecStream && bt.allGated && xs.upHostDev) {
        // Every solve here is a chained job's, so nothing in the head needs
        // the copy: the jobs read their descriptors, inputs and solve rows
        // from the pinned upload over the bus and write the solves' rows and
        // coefficients to the device copy, starting at once (a kernel starts
        // 12-20 us after a copy on its queue): a round's first k_exec 148 ->
        // 118 us after its first copy (profiles/r6m_ge_zero_copy_ab.txt).
        const uint8_t* hd = xs.upHostDev;
        be_launch_ge((const GeDesc*)(hd + bt.oGeD), hd + bt.oGeIn, (uint32_t)bt.nGe, resultsDev,
                     (SolveRow*)(bt.upBase + bt.oSR), bt.upBase + bt.oCoef, bt.geMaxRows, bt.geMaxCols, nullptr,
                     false, (const SolveRow*)(hd + bt.oSR));
        be_side_upload_ingest(bt.upBytes > head ? &rest : nullptr, (const IngestDesc*)(bt.upBase + bt.oIngD),
                              (uint32_t)bt.nIngest, bt.maxIngest, (const uint32_t*)(bt.upBase + bt.oIngB),
                              (uint32_t)bt.nIngBlocks);
        ingested = true;
    } else if (bt.nGe) {
        const BeCopy hc{(uint64_t)(uintptr_t)xs.upDev, (uint64_t)(uintptr_t)xs.upHost, head};
        be_launch_ge((const GeDesc*)(bt.upBase + bt.oGeD), bt.upBase + bt.oGeIn, (uint32_t)bt.nGe, resultsDev,
                     (SolveRow*)(bt.upBase + bt.oSR), bt.upBase + bt.oCoef, bt.geMaxRows, bt.geMaxCols,
                     head ? &hc : nullptr, !(head && kGeOnCodecStream));
        if (head && kGeOnCodecStream) {
            be_side_upload_ingest(bt.upBytes > head ? &rest : nullptr, (const IngestDesc*)(bt.upBase + bt.oIngD),
                                  (uint32_t)bt.nIngest, bt.maxIngest, (const uint32_t*)(bt.upBase + bt.oIngB),
                                  (uint32_t)bt.nIngBlocks);
            ingested = true;
        }
    }
    if (!ingested && copyUp && bt.upBytes > head)
        be_copy_pinned(&rest, 1, true);
    if (!ingested && bt.nIngest)
        be_launch_ingest((const IngestDesc*)(bt.upBase + bt.oIngD), (uint32_t)bt.nIngest, bt.maxIngest,
                         (const uint32_t*)(bt.upBase + bt.oIngB), (uint32_t)bt.nIngBlocks);
    if (xs.acctZero) {
        be_memset(acctDev, 0, 4 * sizeof(uint64_t));
        xs.acctZero = false;
    }
    if (bt.wideZero)
        be_memset(xs.wideDev, 0, xs.wideCap);
    // k_ldpc items of every exec phase before the first solve go in one
    // launch (they read only window elements that exist before the flush's
    // first solve); a phase after a solve launches its own
    size_t wideDone = 0;
    for (size_t k = 0; k < bt.phases.size() && bt.phases[k].kind == Phase::EXEC; ++k)
        wideDone = bt.phases[k].wideBegin + bt.phases[k].wideCount;
    if (wideDone) {
        if (ingested)
            be_join_ge();   // (its items and the elements they read came with the side stream)
        be_launch_ldpc((const LdpcItem*)(bt.upBase + bt.oWide), (uint32_t)wideDone, acctDev + 3);
    }
    // The codec stream joins the matrix jobs before the first executor launch
    // (they run beside k_ingest): joined only before the decoders' phases,
    // they shared the CUs with the encoders' k_exec, which slowed from 87 to
    // 107 us per launch for no gain in the step (same box, interleaved,
    // 4.86 vs 5.04 ms per step: profiles/r6r_ge_join_ab.txt).
    for (const Phase& ph : bt.phases) {
        be_join_ge();   // (no-op once joined)
        if (ph.kind == Phase::EXEC) {
            if (ph.wideCount && ph.wideBegin >= wideDone)
                be_launch_ldpc((const LdpcItem*)(bt.upBase + bt.oWide) + ph.wideBegin, (uint32_t)ph.wideCount,
                               acctDev + 3);
            be_launch_exec(bt.upBase + bt.oStream, (const ExecItem*)(bt.upBase + bt.oItems) + ph.itemBegin,
                           (uint32_t)ph.itemCount, acctDev, resultsDev, ph.maxRows);
            st.execLaunches++;
        } else {
            // solve items index solves globally; pass the global desc base
            be_launch_solve((const SolveDesc*)(bt.upBase + bt.oSD), (const SolveRow*)(bt.upBase + bt.oSR),
                            bt.upBase + bt.oCoef, resultsDev, (const SolveItem*)(bt.upBase + bt.oSI) + ph.itemBegin,
                            (uint32_t)ph.itemCount, ph.maxRows, acctDev + 1, (uint32_t)ph.solveBegin,
                            (uint32_t)ph.solveCount);
        }
    }
    // the counters and solve results, then the downloads, in one call (one
    // kernel when small; its range list was laid out with the upload: a
    // drop-in submission carries a range per application call)
    be_join_ge();
    be_copy_list(bt.copies.data(), xs.downHostDev ? bt.upBase + bt.oCopy : nullptr, (unsigned)bt.copies.size(),
                 false);
    bt.fence = be_fence();
    bt.launched = true;
    std::lock_guard<std::mutex> g(statsMu_);
    flushStats_.add(st);
}

void Engine::completer_loop()
{
    for (;;) {
        Batch* b = nullptr;
        {
            std::unique_lock<std::mutex> lk(qMu_);
            completeCv_.wait(lk, [&] { return stop_ || !toComplete_.empty(); });
            if (stop_)
                return;
            b = toComplete_.front();
            toComplete_.pop_front();
            completing_ = true;
        }
        tl("complete begin", b->ticket);
        // (released buffers go back to the depot tagged with the ticket:
        // refill() takes them only once the ticket reads as done below, so a
        // caller that gathers a completed submission's outputs before its
        // next submission -- the siamese_gpu.h lifetime rule -- always sees
        // that submission done before anyone can reuse its buffers)
        if (complete_batch(*b))
            reclaim_batch(*b);
        tl("complete end", b->ticket);
        // SGPU_TEST_PUBLISH_DELAY_US: widen the window between filing the
        // released buffers and publishing the ticket (CPU test of the rule above)
        static const long kPublishDelayUs = [] {
            const char* v = std::getenv("SGPU_TEST_PUBLISH_DELAY_US");
            return v ? std::atol(v) : 0L;
        }();
        if (kPublishDelayUs > 0)
            std::this_thread::sleep_for(std::chrono::microseconds(kPublishDelayUs));
        {
            // tickets publish in order: an earlier one may still be completing
            // on the thread that flushed it inline
            std::unique_lock<std::mutex> g(qMu_);
            doneCv_.wait(g, [&] { return stop_ || doneTicket_ + 1 >= b->ticket; });
            if (sets_[b->set].busyTicket == b->ticket)   // (a failed batch may never have claimed it)
                sets_[b->set].busyTicket = 0;
            doneTicket_ = b->ticket;
            doneSeen_.store(b->ticket, std::memory_order_release);
            completing_ = false;
        }
        setCv_.notify_all();
        doneCv_.notify_all();
        delete b;
    }
}

bool Engine::complete_batch(Batch& bt)
{
    const uint64_t t0 = now_ns();
    EngineStats st;
    // small flushes (a few instances: single-stream latency) poll the fence
    const size_t bodies = bt.bodies[0].size() + bt.bodies[1].size();
    // (small flushes spin: single-stream latency; mid-size ones take the
    // runtime's blocking wait: the drop-in ABI's group-committed calls;
    // large ones sleep-poll, be_fence_wait)
    const bool ok = bt.launched && be_fence_wait(bt.fence, bodies <= 16 ? 2000u : 0u, bodies > 64) && !failed();
    const uint64_t t1 = now_ns();
    tl("fence passed", bt.ticket);
    st.waitNs = t1 - t0;
    if (!ok) {
        // The results buffer and downloads of this submission are not valid:
        // deliver nothing, keep its released buffers out of reuse, and fail
        // every instance from now on.
        failed_.store(true, std::memory_order_relaxed);
        for (int g = 0; g < 2; ++g)
            for (ProgramBody* p : bt.bodies[g]) {
                p->callbacks.clear();
                ProgramBody::put(p);
            }
        std::lock_guard<std::mutex> g(statsMu_);
        flushStats_.add(st);
        return false;
    }
    XferSet& xs = sets_[bt.set];
    for (const Batch::Download& d : bt.downloads)
        std::memcpy(d.host, xs.downHost + d.off, d.bytes);
    // bytes the kernels counted: terms the executor expanded itself, and the
    // solves' back-substitution (source bytes, recovered bytes); the device
    // counters of a transfer set only grow
    uint64_t acct[4], cur[4];
    std::memcpy(cur, xs.downHost, sizeof(cur));
    for (int k = 0; k < 4; ++k) {
        acct[k] = cur[k] - xs.acctPrev[k];
        xs.acctPrev[k] = cur[k];
    }
    st.refOpBytes += acct[0] + acct[1] + acct[3];
    st.outBytes += acct[2];
    st.solveBytes += acct[1] + acct[2];
    st.ldpcBytes += acct[3];
    const uint32_t* results = (const uint32_t*)(xs.downHost + kAcctBytes);
    for (int g = 0; g < 2; ++g)
        for (size_t i = 0; i < bt.bodies[g].size(); ++i) {
            ProgramBody* p = bt.bodies[g][i];
            for (Completion& fn : p->callbacks)
                fn(results + bt.resultBase[g][i]);
            ProgramBody::put(p);
        }
    st.completeNs = now_ns() - t1;
    std::lock_guard<std::mutex> g(statsMu_);
    flushStats_.add(st);
    return true;
}

void Engine::reclaim_batch(Batch& bt)
{
    const uint64_t t2 = now_ns();
    EngineStats st;
    // Released buffers are free once this submission (and so every earlier
    // one) has run: they go back to the depot as magazines, and the emptied
    // queues back to their shard.
    for (size_t qi = 0; qi < bt.queues.size(); ++qi) {
        Shard::Queues& q = bt.queues[qi];
        for (size_t cls = 0; cls < q.released.size(); ++cls) {
            std::vector<uint8_t*>& r = q.released[cls];
            if (r.empty())
                continue;
            std::lock_guard<std::mutex> g(depotMu_);
            if (cls >= depot_.size())
                depot_.resize(cls + 1);
            if (r.size() <= kMaxMagazine) {
                depot_[cls].emplace_back();
                depot_[cls].back().ticket = bt.ticket;
                depot_[cls].back().bufs.swap(r);
            } else {
                for (size_t k = 0; k < r.size(); k += kMaxMagazine) {
                    depot_[cls].emplace_back();
                    depot_[cls].back().ticket = bt.ticket;
                    depot_[cls].back().bufs.assign(r.begin() + (long)k,
                                                   r.begin() + (long)std::min(r.size(), k + kMaxMagazine));
                }
                r.clear();
            }
        }
        q.clear();
        Shard* s = bt.queueOwner[qi];
        std::lock_guard<std::mutex> g(s->mu);
        if (s->spare.size() < 4)
            s->spare.push_back(std::move(q));
    }
    st.reclaimNs = now_ns() - t2;
    std::lock_guard<std::mutex> g(statsMu_);
    flushStats_.add(st);
}

bool Engine::stage_in(void* dst, const void* src, size_t bytes)
{
    if (failed())
        return false;
    void* m = be_stage_h2d(dst, src, bytes);
    if (!m)
        return false;
    std::lock_guard<std::mutex> g(qMu_);
    pendingMarks_.push_back(m);
    return true;
}

bool Engine::gather_land(GatherSlot& g)
{
    if (!g.landed)
        return true;
    void* m = g.landed;
    g.landed = nullptr;
    if (!be_mark_sync(m)) {
        failed_.store(true, std::memory_order_relaxed);
        return false;
    }
    return true;
}

int64_t Engine::gather_async(unsigned count, const void* const* srcs, const unsigned* bytes,
                             void* pinnedOut)
{
    return gather_async_framed(count, srcs, bytes, nullptr, nullptr, pinnedOut);
}

int64_t Engine::gather_async_framed(unsigned count, const void* const* srcs, const unsigned* bytes,
                                    const uint8_t* hdrs, const unsigned* hdrLens, void* pinnedOut)
{
    if (failed())
        return -1;
    std::lock_guard<std::mutex> lk(gatherMu_);
    const int64_t ticket = ++gNext_;
    if (count == 0)
        return ticket;
    GatherSlot& g = gslots_[ticket % kGatherSlots];
    if (!gather_land(g))   // (the slot's previous gather, kGatherSlots back)
        return -1;
    const size_t upBytes = count * sizeof(IngestDesc);
    size_t total = 0;
    for (unsigned i = 0; i < count; ++i)
        total = align16(total + bytes[i] + (hdrLens ? hdrLens[i] : 0));
    auto grow = [](uint8_t*& h, uint8_t*& d, size_t& cap, size_t need, bool host) {
        if (need <= cap)
            return;
        size_t c = cap ? cap : (1u << 20);
        while (c < need)
            c *= 2;
        if (h)
            be_host_free(h);
        if (d)
            be_dev_free(d);
        h = host ? (uint8_t*)be_host_alloc(c) : nullptr;
        d = (uint8_t*)be_dev_alloc(c);
        cap = c;
    };
    uint8_t* noHost = nullptr;
    grow(g.upHost, g.upDev, g.upCap, upBytes, true);
    grow(noHost, g.stage, g.stageCap, total, false);
    if (!g.upHost || !g.upDev || !g.stage)
        return -1;
    IngestDesc* descs = reinterpret_cast<IngestDesc*>(g.upHost);
    size_t off = 0;
    for (unsigned i = 0; i < count; ++i) {
        std::memset(&descs[i], 0, sizeof(IngestDesc));
        descs[i].src = (uint64_t)(uintptr_t)srcs[i];
        descs[i].bytes = bytes[i];
        descs[i].dst = (uint64_t)(uintptr_t)g.stage + off;
        if (hdrLens) {
            descs[i].hdrLen = hdrLens[i] < 8 ? hdrLens[i] : 8;
            std::memcpy(descs[i].hdr, hdrs + 8 * (size_t)i, descs[i].hdrLen);
        }
        off = align16(off + bytes[i] + descs[i].hdrLen);
    }
    void* packed = nullptr;
    if (!be_gather(descs, g.upDev, count, g.stage, pinnedOut, total, &packed, &g.landed)) {
        failed_.store(true, std::memory_order_relaxed);
        return -1;
    }
    g.ticket = ticket;
    // later submissions may overwrite the sources (recycled buffers, the
    // next encode's packet): their device work waits for the packing
    std::lock_guard<std::mutex> q(qMu_);
    pendingMarks_.push_back(packed);
    return ticket;
}

bool Engine::gather_wait(int64_t ticket)
{
    std::lock_guard<std::mutex> lk(gatherMu_);
    bool ok = true;
    for (GatherSlot& g : gslots_)
        if (g.landed && g.ticket <= ticket)
            ok = gather_land(g) && ok;
    return ok && !failed();
}

bool Engine::gather_completed(unsigned count, const void* const* srcs, const unsigned* bytes,
                              void* pinnedOut)
{
    const int64_t t = gather_async(count, srcs, bytes, pinnedOut);
    return t > 0 && gather_wait(t);
}

bool Engine::gather(unsigned count, const void* const* srcs, const unsigned* bytes, void* hostOut)
{
    if (!sync())
        return false;
    if (count == 0)
        return true;
    std::vector<IngestDesc> descs(count);
    size_t total = 0;
    for (unsigned i = 0; i < count; ++i) {
        std::memset(&descs[i], 0, sizeof(IngestDesc));
        descs[i].src = (uint64_t)(uintptr_t)srcs[i];
        descs[i].bytes = bytes[i];
        descs[i].dst = total; // offset for now
        total = align16(total + bytes[i]);
    }
    const size_t upBytes = count * sizeof(IngestDesc);
    auto grow = [](uint8_t*& h, uint8_t*& d, size_t& cap, size_t need) {
        if (need <= cap)
            return;
        size_t c = cap ? cap : (1u << 20);
        while (c < need)
            c *= 2;
        if (h)
            be_host_free(h);
        if (d)
            be_dev_free(d);
        h = (uint8_t*)be_host_alloc(c);
        d = (uint8_t*)be_dev_alloc(c);
        cap = c;
    };
    grow(gUpHost_, gUpDev_, gUpCap_, upBytes);
    grow(gHost_, gDev_, gCap_, total);
    for (IngestDesc& d : descs)
        d.dst += (uint64_t)(uintptr_t)gDev_;
    std::memcpy(gUpHost_, descs.data(), upBytes);
    be_h2d(gUpDev_, gUpHost_, upBytes);
    uint32_t maxBytes = 0;
    for (unsigned i = 0; i < count; ++i)
        maxBytes = std::max(maxBytes, bytes[i]);
    be_launch_ingest((const IngestDesc*)gUpDev_, count, maxBytes);
    be_d2h(gHost_, gDev_, total);
    const bool ok = be_sync();
    if (!ok) {
        failed_.store(true, std::memory_order_relaxed);
        return false;
    }
    // unpack the 16-byte-aligned staging layout into the caller's buffer,
    // in parallel chunks (this is the D2H leg of end-to-end packet flows)
    constexpr unsigned kChunk = 2048;
    std::vector<size_t> outOff((count + kChunk - 1) / kChunk + 1), inOff(outOff.size());
    size_t o = 0, in = 0;
    for (unsigned i = 0; i < count; ++i) {
        if (i % kChunk == 0) {
            outOff[i / kChunk] = o;
            inOff[i / kChunk] = in;
        }
        o += bytes[i];
        in = align16(in + bytes[i]);
    }
    pool().run((count + kChunk - 1) / kChunk, [&](size_t c) {
        uint8_t* out = (uint8_t*)hostOut + outOff[c];
        size_t off = inOff[c];
        const unsigned end = std::min<unsigned>(count, (unsigned)(c + 1) * kChunk);
        for (unsigned i = (unsigned)c * kChunk; i < end; ++i) {
            std::memcpy(out, gHost_ + off, bytes[i]);
            out += bytes[i];
            off = align16(off + bytes[i]);
        }
    });
    return ok;
}

} // namespace sgpu
