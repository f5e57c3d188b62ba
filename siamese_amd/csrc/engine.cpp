// engine.cpp -- arena, programs and flush (see engine.h).
#include "engine.h"
#include "backend.h"
#include "pool.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstddef>
#include <cstring>

// dispatch each exec phase's segments longest op list first (see flush)
#ifndef SGPU_EXEC_LPT
#define SGPU_EXEC_LPT 1
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
    assembleNs += o.assembleNs;
    waitNs += o.waitNs;
    completeNs += o.completeNs;
    reclaimNs += o.reclaimNs;
    execLaunches += o.execLaunches;
}

namespace {

uint64_t now_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

} // namespace

// ---------------------------------------------------------------------------
// Program

std::vector<Program::Store>& Program::spare_stores()
{
    thread_local std::vector<Store> spare;
    return spare;
}

void Program::take_store()
{
    std::vector<Store>& spare = spare_stores();
    if (spare.empty())
        return;
    Store& st = spare.back();
    segs_.swap(st.segs);
    rb_.win.swap(st.win);
    rb_.updates.swap(st.updates);
    rb_.rows.swap(st.rows);
    spare.pop_back();
}

void Program::stash_store()
{
    std::vector<Store>& spare = spare_stores();
    if (spare.size() >= 4096)
        return;
    for (Segment& g : segs_) {
        g.ops.clear();
        g.terms.clear();
        g.rowsData.clear();
    }
    rb_.win.clear();
    rb_.updates.clear();
    rb_.rows.clear();
    spare.emplace_back();
    Store& st = spare.back();
    st.segs.swap(segs_);
    st.win.swap(rb_.win);
    st.updates.swap(rb_.updates);
    st.rows.swap(rb_.rows);
}

Program::~Program()
{
    if (!shard_) {
        stash_store();
        return;
    }
    rows_close();
    // The instance goes away with work still queued (e.g. an encoder freed
    // right after its last recovery packet was handed to a decoder, whose
    // copy op lives in this program).  The queued ops still run: hand them
    // to an orphan program the engine deletes after the next flush.  The
    // buffers they touch were released by the instance and are not reused
    // before that flush completes.
    Program* orphan = new Program(eng_, group_);
    orphan->shard_ = shard_;
    orphan->resultWords_ = resultWords_;
    orphan->nsegs_ = nsegs_;
    orphan->segs_.swap(segs_);
    orphan->solves_.swap(solves_);
    orphan->callbacks_.swap(callbacks_);
    orphan->group_ = group_ | 2;   // bit 1: delete after flush
    std::lock_guard<std::mutex> g(shard_->mu);
    auto it = std::find(shard_->dirty.begin(), shard_->dirty.end(), this);
    if (it != shard_->dirty.end())
        *it = orphan;
}

void Program::attach()
{
    Shard& s = eng_->shard();
    shard_ = &s;
    std::lock_guard<std::mutex> g(s.mu);
    s.dirty.push_back(this);
}

void Program::new_segment()
{
    rows_close();
    if (nsegs_ == segs_.size())
        segs_.emplace_back();
    Segment& s = segs_[nsegs_++];
    s.ops.clear();
    s.terms.clear();
    s.rowsData.clear();
    s.rowsWords = 0;
    s.maxExtent = 0;
}

void Program::reset_after_flush()
{
    for (size_t k = 0; k < nsegs_; ++k) {
        segs_[k].ops.clear();
        segs_[k].terms.clear();
        segs_[k].rowsData.clear();
        segs_[k].rowsWords = 0;
        segs_[k].maxExtent = 0;
    }
    nsegs_ = 0;
    solves_.clear();
    callbacks_.clear();
    resultWords_ = 0;
    shard_ = nullptr;
}

void Program::lc_begin(uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix)
{
    touch();
    rows_close();
    if (nsegs_ == 0)
        new_segment();
    Segment& s = segs_[nsegs_ - 1];
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
    Segment& s = segs_[nsegs_ - 1];
    GfOp& op = s.ops.back();
    // An op that keeps all of dst and adds nothing is a no-op.
    if (op.termCount == 0 && op.valid >= op.n) {
        s.ops.pop_back();
        return;
    }
    if (op.n > s.maxExtent)
        s.maxExtent = op.n;
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
    rows_close();
    if (nsegs_ == 0)
        new_segment();
    Segment& s = segs_[nsegs_ - 1];
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
    IngestDesc d;
    std::memset(&d, 0, sizeof(d));
    d.dst = dst.addr();
    d.src = src;
    d.bytes = bytes;
    d.hdrLen = hdrLen;
    std::memcpy(d.hdr, hdr, hdrLen);
    eng_->add_ingest(d, -1);
}

uint32_t Program::solve(const std::vector<SolveRow>& rows, const uint8_t* coef, uint32_t maxBytes)
{
    touch();
    if (nsegs_ == 0)
        new_segment(); // the segment preceding this solve
    PendingSolve ps;
    std::memset(&ps.desc, 0, sizeof(ps.desc));
    ps.desc.m = (uint32_t)rows.size();
    ps.desc.maxBytes = maxBytes;
    ps.desc.result = resultWords_;
    resultWords_ += ps.desc.m + 1;
    ps.rows = rows;
    ps.coef.assign(coef, coef + rows.size() * rows.size());
    const uint32_t r = ps.desc.result;
    solves_.push_back(std::move(ps));
    new_segment(); // ops after the solve go to the next segment
    return r;
}

void Program::on_complete(Completion fn)
{
    touch();
    callbacks_.push_back(std::move(fn));
}

// ---- Siamese row batches ---------------------------------------------------

void Program::rows_open(uint32_t base, bool keepWindow)
{
    RowsBuild& b = rb_;
    rows_close();
    touch();
    if (nsegs_ == 0)
        new_segment();
    b.open = true;
    b.haveSums = false;
    b.readMask = 0;
    if (!keepWindow) {
        b.base = base;
        b.win.clear();
    }
    b.updates.clear();
    for (int& u : b.updateOf)
        u = -1;
    b.rows.clear();
    b.maxExtent = 0;
}

WinEntry* Program::rows_window(uint32_t lo, uint32_t hi, uint32_t* from)
{
    RowsBuild& b = rb_;
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
    RowsBuild& b = rb_;
    // a row of this batch already read sum k: the update belongs to a new
    // batch over the same window (its rows run after this batch's rows)
    if (b.readMask >> k & 1)
        rows_open(b.base, true);
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
    b.updateOf[k] = (int)b.updates.size();
    b.updates.push_back(u);
    if (n > b.maxExtent)
        b.maxExtent = n;
}

void Program::rows_row(const WinEntry* sums, uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix,
                       uint32_t mask0, uint32_t mask1, unsigned row, uint32_t ldpcN,
                       uint32_t ldpcFirst, const uint8_t* lit, uint32_t litLen)
{
    RowsBuild& b = rb_;
    if (b.haveSums && std::memcmp(b.sums, sums, sizeof(b.sums)) != 0)
        rows_open(b.base, true);
    if (!b.haveSums) {
        std::memcpy(b.sums, sums, sizeof(b.sums));
        b.haveSums = true;
    }
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
    if (copies_.empty()) {
        rows_close();
        if (nsegs_ == 0)
            new_segment();
    }
    CopyItem c;
    std::memset(&c, 0, sizeof(c));
    c.dst = dst;
    c.src = src;
    c.len = len;
    copies_.push_back(c);
    Segment& g = segs_[nsegs_ - 1];
    if (len > g.maxExtent)
        g.maxExtent = len;
}

void Program::rows_close()
{
    if (!copies_.empty()) {
        // seal the open copy batch
        Segment& g = segs_[nsegs_ - 1];
        GfOp op;
        std::memset(&op, 0, sizeof(op));
        op.kind = OP_COPIES;
        op.n = (uint32_t)copies_.size();
        op.termBegin = (uint32_t)(g.rowsData.size() / 16);
        op.termCount = (uint32_t)copies_.size() * kCopyWords;
        g.ops.push_back(op);
        const size_t at = g.rowsData.size();
        g.rowsData.resize(at + copies_.size() * sizeof(CopyItem));
        std::memcpy(g.rowsData.data() + at, copies_.data(), copies_.size() * sizeof(CopyItem));
        g.rowsWords += op.termCount;
        copies_.clear();
    }
    RowsBuild& b = rb_;
    if (!b.open)
        return;
    b.open = false;
    if (b.rows.empty() && b.updates.empty())
        return;
    if (!b.haveSums)
        std::memset(b.sums, 0, sizeof(b.sums));
    Segment& s = segs_[nsegs_ - 1];
    const uint32_t E = (uint32_t)b.win.size();
    const uint32_t U = (uint32_t)b.updates.size();
    const uint32_t R = (uint32_t)b.rows.size();
    const uint32_t words = kRowSums + E + U * kUpdateWords + R * kRowWords;
    GfOp op;
    std::memset(&op, 0, sizeof(op));
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
    s.rowsWords += words;
    if (b.maxExtent > s.maxExtent)
        s.maxExtent = b.maxExtent;
}

// ---------------------------------------------------------------------------
// Engine: shards, arena, statistics

Engine* Engine::global()
{
    static Engine e;
    return &e;
}

Engine::~Engine() = default;

bool Engine::init(int device, const char** err)
{
    if (ready_)
        return true;
    if (!be_init(device, err))
        return false;
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
    if (!pool_)
        pool_.reset(new WorkerPool(WorkerPool::default_threads()));
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
    EngineStats t = flushStats_;
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

namespace {

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

size_t cap_class(uint32_t cap)
{
    if (cap <= 4096)
        return cap / 64 - 1;                 // 0..63
    if (cap <= 131072)
        return 64 + cap / 1024 - 5;          // 64..187
    return 188 + cap / 65536 - 3;
}

} // namespace

namespace {
constexpr size_t kChunkBytes = 64u << 20;    // one hipMalloc
constexpr size_t kRegionBytes = 4u << 20;    // a shard's bump region
constexpr size_t kMagazine = 512;            // buffers moved per depot transfer
constexpr size_t kKeepFree = 8 * kMagazine;  // free buffers of a class a shard keeps through a reclaim
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
        uint8_t* base = (uint8_t*)be_dev_alloc(kChunkBytes);
        if (!base)
            return nullptr;
        arenaBytes_ += kChunkBytes;
        chunks_.push_back(Chunk{base, kChunkBytes, 0});
    }
    Chunk& c = chunks_.back();
    uint8_t* p = c.base + c.used;
    c.used += bytes;
    return p;
}

// Refill shard s's empty list of class `cls`: a magazine from the depot if
// one is there, otherwise fresh buffers cut from the shard's bump region.
bool Engine::refill(Shard& s, size_t cls, uint32_t cap)
{
    std::vector<uint8_t*>& list = s.freeLists[cls];
    {
        std::lock_guard<std::mutex> g(depotMu_);
        if (cls < depot_.size() && !depot_[cls].empty()) {
            std::vector<uint8_t*>& d = depot_[cls];
            const size_t take = std::min(kMagazine, d.size());
            list.insert(list.end(), d.end() - take, d.end());
            d.resize(d.size() - take);
            return true;
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

// Return surplus free buffers of shard s to the depot in magazines.
void Engine::spill(Shard& s)
{
    for (size_t cls = 0; cls < s.freeLists.size(); ++cls) {
        std::vector<uint8_t*>& list = s.freeLists[cls];
        if (list.size() <= kKeepFree + kMagazine)
            continue;
        const size_t keep = kKeepFree;
        std::lock_guard<std::mutex> g(depotMu_);
        if (cls >= depot_.size())
            depot_.resize(cls + 1);
        depot_[cls].insert(depot_[cls].end(), list.begin() + keep, list.end());
        list.resize(keep);
    }
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

void Engine::release(DevBuf& b)
{
    if (b.ptr) {
        Shard& s = shard();
        s.pendingFree.push_back(b);
        s.inUse -= b.cap;
    }
    b = DevBuf();
}

void Engine::download(void* hostDst, uint64_t devSrc, uint32_t bytes)
{
    if (bytes)
        shard().downloads.push_back(Shard::Download{hostDst, devSrc, bytes});
}

void Engine::stage_host_ingest(const DevBuf& dst, const void* data, uint32_t bytes,
                               const uint8_t* hdr, uint32_t hdrLen)
{
    // Stage hdr || data contiguously so the device copy is aligned.
    Shard& s = shard();
    const size_t off = (s.hostStage.size() + 15) & ~(size_t)15;
    s.hostStage.resize(off + hdrLen + bytes);
    std::memcpy(s.hostStage.data() + off, hdr, hdrLen);
    std::memcpy(s.hostStage.data() + off + hdrLen, data, bytes);
    IngestDesc d;
    std::memset(&d, 0, sizeof(d));
    d.dst = dst.addr();
    d.src = 0;
    d.bytes = hdrLen + bytes;
    d.hdrLen = 0;
    add_ingest(d, (int64_t)off);
}

void Engine::add_ingest(const IngestDesc& d, int64_t hostStageOffset)
{
    Shard& s = shard();
    s.ingest.push_back(Shard::IngestRec{d, hostStageOffset});
}

bool Engine::pending() const
{
    std::lock_guard<std::mutex> g(shardsMu_);
    for (const auto& s : shards_)
        if (!s->dirty.empty() || !s->ingest.empty() || !s->downloads.empty())
            return true;
    return false;
}

void Engine::ensure_up(size_t bytes)
{
    if (bytes <= upCap_)
        return;
    size_t cap = upCap_ ? upCap_ : (1u << 20);
    while (cap < bytes)
        cap *= 2;
    if (upHost_)
        be_host_free(upHost_);
    if (upDev_)
        be_dev_free(upDev_);
    upHost_ = (uint8_t*)be_host_alloc(cap);
    upDev_ = (uint8_t*)be_dev_alloc(cap);
    upCap_ = cap;
}

void Engine::ensure_down(size_t bytes)
{
    if (bytes <= downCap_)
        return;
    size_t cap = downCap_ ? downCap_ : (1u << 20);
    while (cap < bytes)
        cap *= 2;
    if (downHost_)
        be_host_free(downHost_);
    if (downDev_)
        be_dev_free(downDev_);
    downHost_ = (uint8_t*)be_host_alloc(cap);
    downDev_ = (uint8_t*)be_dev_alloc(cap);
    downCap_ = cap;
}

// ---------------------------------------------------------------------------
// Engine: flush
//
// 1. A sequential pass over the queued programs fixes every segment's place
//    in the upload (ops, terms, work items) and every solve's place in the
//    result array.
// 2. The pool copies segments, ingest descriptors and staged host payloads
//    into the pinned upload buffer in parallel.
// 3. One H2D copy, then ingest, executor and solve launches in phase order.

namespace {

inline size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

struct Phase
{
    enum Kind { EXEC, SOLVE } kind;
    size_t itemBegin, itemCount;    // exec items or solve items
    size_t solveBegin, solveCount;  // solve descs (SOLVE)
    uint32_t maxRows;               // largest m among them (SOLVE)
};

struct SegRef
{
    Program* prog;
    uint32_t seg;
    uint32_t wordBase, words, itemBase;
};

struct ShardRef
{
    Shard* shard;
    size_t descBase, stageBase;
};

} // namespace

bool Engine::flush()
{
    if (flight_.active && !sync())
        return false;
    if (failed())
        return false;

    std::vector<Shard*> shards;
    {
        std::lock_guard<std::mutex> g(shardsMu_);
        for (auto& s : shards_)
            shards.push_back(s.get());
    }
    bool any = false;
    for (Shard* s : shards)
        any = any || !s->dirty.empty() || !s->ingest.empty() || !s->downloads.empty() ||
              !s->pendingFree.empty();
    if (!any)
        return true;
    const uint64_t t0 = now_ns();

    // ---- 1. layout -----------------------------------------------------------
    std::vector<Program*> progs[2];
    for (Shard* s : shards)
        for (Program* p : s->dirty)
            progs[p->group_ & 1].push_back(p);
    // seal every open Siamese row batch (serialises its table and rows)
    for (int g = 0; g < 2; ++g)
        pool().run(progs[g].size(), [&](size_t i) { progs[g][i]->rows_close(); });

    uint32_t resultWords = 0;
    std::vector<uint32_t> resultBase[2];
    for (int g = 0; g < 2; ++g)
        for (Program* p : progs[g]) {
            resultBase[g].push_back(resultWords);
            resultWords += p->resultWords_;
        }

    std::vector<SegRef> segs;
    std::vector<Phase> phases;
    std::vector<SolveDesc> sdescs;
    // solve rows and coefficients are copied straight into the upload by the
    // assembly tasks (SolveRef: where each pending solve's data goes)
    struct SolveRef
    {
        const Program::PendingSolve* ps;
        size_t rowBase, coefBase;
    };
    std::vector<SolveRef> srefsSolve;
    size_t nSolveRows = 0, nCoef = 0;
    std::vector<SolveItem> sitems;
    size_t nOps = 0, nTerms = 0, nWords = 0, nItems = 0;
    for (int g = 0; g < 2; ++g) {
        size_t maxSegs = 0;
        for (Program* p : progs[g])
            maxSegs = std::max(maxSegs, p->nsegs_);
        for (size_t k = 0; k < maxSegs; ++k) {
            Phase ex{Phase::EXEC, nItems, 0, 0, 0, 0};
            const size_t segBegin = segs.size();
            for (Program* p : progs[g]) {
                if (k >= p->nsegs_)
                    continue;
                const Program::Segment& s = p->segs_[k];
                if (s.ops.empty())
                    continue;
                const size_t words = kOpWords * s.ops.size() + s.terms.size() + s.rowsWords;
                segs.push_back(SegRef{p, (uint32_t)k, (uint32_t)nWords, (uint32_t)words,
                                      (uint32_t)nItems});
                nOps += s.ops.size();
                nTerms += s.terms.size();
                nWords += words;
                nItems += (s.maxExtent + kExecTileBytes - 1) / kExecTileBytes;
            }
#if SGPU_EXEC_LPT
            // Longest op lists first: workgroups are dispatched in blockIdx
            // order and a launch runs in about two rounds of one workgroup per
            // CU, so the short segments fill the second round's tail.
            {
                std::vector<uint32_t> order(segs.size() - segBegin);
                for (uint32_t i = 0; i < order.size(); ++i)
                    order[i] = i;
                std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
                    return segs[segBegin + a].words > segs[segBegin + b].words;
                });
                uint32_t ib = (uint32_t)ex.itemBegin;
                for (uint32_t i : order) {
                    SegRef& r = segs[segBegin + i];
                    r.itemBase = ib;
                    ib += (r.prog->segs_[r.seg].maxExtent + kExecTileBytes - 1) / kExecTileBytes;
                }
            }
#endif
            ex.itemCount = nItems - ex.itemBegin;
            if (ex.itemCount)
                phases.push_back(ex);

            Phase sv{Phase::SOLVE, sitems.size(), 0, sdescs.size(), 0, 0};
            for (size_t pi = 0; pi < progs[g].size(); ++pi) {
                Program* p = progs[g][pi];
                if (k >= p->solves_.size())
                    continue;
                const Program::PendingSolve& ps = p->solves_[k];
                SolveDesc d = ps.desc;
                d.result += resultBase[g][pi];
                d.rowBegin = (uint32_t)nSolveRows;
                d.coefOffset = nCoef;
                srefsSolve.push_back(SolveRef{&ps, nSolveRows, nCoef});
                nSolveRows += ps.rows.size();
                nCoef += ps.coef.size();
                const uint32_t sidx = (uint32_t)sdescs.size();
                sdescs.push_back(d);
                sv.maxRows = std::max(sv.maxRows, d.m);
                for (uint32_t t = 0; t < d.maxBytes; t += kTileBytes)
                    sitems.push_back(SolveItem{sidx, t});
            }
#if SGPU_EXEC_LPT
            // largest solves first (the serial pivot chain grows with m)
            std::stable_sort(sitems.begin() + sv.itemBegin, sitems.end(),
                             [&](const SolveItem& a, const SolveItem& b) {
                                 return sdescs[a.solve].m > sdescs[b.solve].m;
                             });
#endif
            sv.itemCount = sitems.size() - sv.itemBegin;
            sv.solveCount = sdescs.size() - sv.solveBegin;
            if (sv.solveCount)
                phases.push_back(sv);
        }
    }

    std::vector<ShardRef> srefs;
    size_t nIngest = 0, stageBytes = 0;
    for (Shard* s : shards) {
        srefs.push_back(ShardRef{s, nIngest, stageBytes});
        nIngest += s->ingest.size();
        stageBytes = align16(stageBytes + s->hostStage.size());
    }

    size_t off = 0;
    const size_t oStage = off;
    off = align16(off + stageBytes);
    const size_t oIngD = off;
    off = align16(off + nIngest * sizeof(IngestDesc));
    const size_t oStream = off;
    off = align16(off + nWords * 16);
    const size_t oItems = off;
    off = align16(off + nItems * sizeof(ExecItem));
    const size_t oSD = off;
    off = align16(off + sdescs.size() * sizeof(SolveDesc));
    const size_t oSR = off;
    off = align16(off + nSolveRows * sizeof(SolveRow));
    const size_t oCoef = off;
    off = align16(off + nCoef);
    const size_t oSI = off;
    off = align16(off + sitems.size() * sizeof(SolveItem));
    const size_t upBytes = off;
    if (upBytes)
        ensure_up(upBytes);

    // ---- 2. parallel assembly into the pinned upload buffer ----------------
    uint8_t* up = upHost_;
    const uint64_t stageDev = (uint64_t)(uintptr_t)(upDev_ + oStage);
    constexpr size_t kIngestChunk = 16384;
    constexpr size_t kSolveChunk = 64;
    struct Task
    {
        int kind;   // 0 = segment, 1 = ingest chunk, 2 = solve chunk
        size_t a, b;
    };
    std::vector<Task> tasks;
    for (size_t i = 0; i < segs.size(); ++i)
        tasks.push_back(Task{0, i, 0});
    for (size_t i = 0; i < srefsSolve.size(); i += kSolveChunk)
        tasks.push_back(Task{2, i, 0});
    for (size_t si = 0; si < srefs.size(); ++si)
        for (size_t c = 0; c < srefs[si].shard->ingest.size(); c += kIngestChunk)
            tasks.push_back(Task{1, si, c});
    pool().run(tasks.size(), [&](size_t ti) {
        const Task& t = tasks[ti];
        if (t.kind == 0) {
            const SegRef& r = segs[t.a];
            const Program::Segment& s = r.prog->segs_[r.seg];
            uint8_t* w = up + oStream + (size_t)r.wordBase * 16;
            for (const GfOp& op : s.ops) {
                if (op.kind == OP_ROWS || op.kind == OP_COPIES) {
                    std::memcpy(w, &op, sizeof(GfOp));
                    w += sizeof(GfOp);
                    const size_t bytes = (size_t)op.termCount * 16;   // block (rows_close)
                    std::memcpy(w, s.rowsData.data() + (size_t)op.termBegin * 16, bytes);
                    w += bytes;
                    continue;
                }
                std::memcpy(w, &op, sizeof(GfOp));
                w += sizeof(GfOp);
                if (op.kind == OP_LINCOMB && op.termCount) {
                    const size_t bytes = (size_t)op.termCount * sizeof(GfTerm);
                    std::memcpy(w, s.terms.data() + op.termBegin, bytes);
                    w += bytes;
                }
            }
            ExecItem* items = (ExecItem*)(up + oItems) + r.itemBase;
            const uint32_t nItems = (uint32_t)s.ops.size();
            uint32_t n = 0;
            for (uint32_t tb = 0; tb < s.maxExtent; tb += kExecTileBytes)
                items[n++] = ExecItem{r.wordBase, r.words, nItems, tb};
        } else if (t.kind == 2) {
            const size_t end = std::min(srefsSolve.size(), t.a + kSolveChunk);
            for (size_t i = t.a; i < end; ++i) {
                const SolveRef& r = srefsSolve[i];
                std::memcpy(up + oSR + r.rowBase * sizeof(SolveRow), r.ps->rows.data(),
                            r.ps->rows.size() * sizeof(SolveRow));
                std::memcpy(up + oCoef + r.coefBase, r.ps->coef.data(), r.ps->coef.size());
            }
        } else {
            const ShardRef& sr = srefs[t.a];
            const Shard& s = *sr.shard;
            const size_t end = std::min(s.ingest.size(), t.b + kIngestChunk);
            IngestDesc* descs = (IngestDesc*)(up + oIngD) + sr.descBase;
            for (size_t i = t.b; i < end; ++i) {
                IngestDesc d = s.ingest[i].d;
                if (s.ingest[i].hostOffset >= 0)
                    d.src = stageDev + sr.stageBase + (uint64_t)s.ingest[i].hostOffset;
                descs[i] = d;
            }
            if (t.b == 0 && !s.hostStage.empty())
                std::memcpy(up + oStage + sr.stageBase, s.hostStage.data(), s.hostStage.size());
        }
    });
    if (!sdescs.empty()) {
        std::memcpy(up + oSD, sdescs.data(), sdescs.size() * sizeof(SolveDesc));
        std::memcpy(up + oSI, sitems.data(), sitems.size() * sizeof(SolveItem));
    }

    // download area: the executor's byte counter (kAcctBytes), the solve
    // results, then each requested range
    constexpr size_t kAcctBytes = 16;
    size_t dOff = align16(kAcctBytes + (size_t)resultWords * 4);
    flight_.downloads.clear();
    std::vector<Shard::Download> dls;
    for (Shard* s : shards)
        for (const Shard::Download& d : s->downloads) {
            flight_.downloads.push_back(InFlight::Download{d.host, dOff, d.bytes});
            dls.push_back(d);
            dOff = align16(dOff + d.bytes);
        }
    ensure_down(dOff);

    // ---- 3. launch -----------------------------------------------------------
    if (upBytes)
        be_h2d(upDev_, upHost_, upBytes);
    if (nIngest)
        be_launch_ingest((const IngestDesc*)(upDev_ + oIngD), (uint32_t)nIngest);
    uint64_t* acctDev = (uint64_t*)downDev_;
    uint32_t* resultsDev = (uint32_t*)(downDev_ + kAcctBytes);
    be_memset(acctDev, 0, sizeof(uint64_t));
    for (const Phase& ph : phases) {
        if (ph.kind == Phase::EXEC) {
            be_launch_exec(upDev_ + oStream, (const ExecItem*)(upDev_ + oItems) + ph.itemBegin,
                           (uint32_t)ph.itemCount, acctDev);
            flushStats_.execLaunches++;
        } else {
            const SolveDesc* sd = (const SolveDesc*)(upDev_ + oSD) + ph.solveBegin;
            be_launch_solve_prefix(sd, (const SolveRow*)(upDev_ + oSR), upDev_ + oCoef, resultsDev,
                                   (uint32_t)ph.solveCount);
            // solve items index solves globally; pass the global desc base
            be_launch_solve_main((const SolveDesc*)(upDev_ + oSD), (const SolveRow*)(upDev_ + oSR),
                                 upDev_ + oCoef, resultsDev,
                                 (const SolveItem*)(upDev_ + oSI) + ph.itemBegin,
                                 (uint32_t)ph.itemCount, ph.maxRows);
        }
    }
    be_d2h(downHost_, downDev_, kAcctBytes + (size_t)resultWords * 4);
    for (size_t i = 0; i < dls.size(); ++i)
        be_d2h(downHost_ + flight_.downloads[i].off, (const void*)(uintptr_t)dls[i].dev,
               dls[i].bytes);

    // ---- bookkeeping -----------------------------------------------------------
    flushStats_.flushes++;
    flushStats_.launches += phases.size() + (nIngest ? 1 : 0);
    flushStats_.ops += nOps;
    flushStats_.terms += nTerms;
    flushStats_.solves += sdescs.size();
    flushStats_.ingests += nIngest;
    flushStats_.uploadBytes += upBytes;
    flushStats_.assembleNs += now_ns() - t0;

    flight_.callbacks.clear();
    for (int g = 0; g < 2; ++g)
        for (size_t pi = 0; pi < progs[g].size(); ++pi) {
            Program* p = progs[g][pi];
            if (!p->callbacks_.empty()) {
                flight_.callbacks.emplace_back();
                flight_.callbacks.back().first = resultBase[g][pi];
                flight_.callbacks.back().second.swap(p->callbacks_);
            }
            if (p->group_ & 2)
                delete p;   // orphan of a freed instance (see ~Program)
            else
                p->reset_after_flush();
        }
    flight_.active = true;
    for (Shard* s : shards) {
        s->dirty.clear();
        s->ingest.clear();
        s->hostStage.clear();
        s->downloads.clear();
        // buffers released before this flush may be reused once it completes
        s->flightFree.swap(s->pendingFree);
        s->pendingFree.clear();
    }
    return true;
}

bool Engine::gather(unsigned count, const void* const* srcs, const unsigned* bytes, void* hostOut)
{
    if (flight_.active && !sync())
        return false;
    if (failed())
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
    be_launch_ingest((const IngestDesc*)gUpDev_, count);
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

bool Engine::sync()
{
    if (!flight_.active)
        return true;
    const uint64_t t0 = now_ns();
    const bool ok = be_sync();
    if (!ok) {
        // The results buffer and downloads of this flush are not valid:
        // deliver nothing, keep the flush's released buffers out of reuse,
        // and fail every instance from now on.
        failed_.store(true, std::memory_order_relaxed);
        flight_.callbacks.clear();
        flight_.downloads.clear();
        flight_.active = false;
        flushStats_.waitNs += now_ns() - t0;
        return false;
    }
    for (const InFlight::Download& d : flight_.downloads)
        std::memcpy(d.host, downHost_ + d.off, d.bytes);
    const uint64_t t1 = now_ns();
    // Completions of different programs touch different instances: run them
    // in parallel, each program's in order.
    // bytes the executor counted for the terms it expanded itself
    uint64_t acct = 0;
    std::memcpy(&acct, downHost_, sizeof(acct));
    flushStats_.refOpBytes += acct;
    const uint32_t* results = (const uint32_t*)(downHost_ + 16);
    pool().run(flight_.callbacks.size(), [&](size_t i) {
        auto& cb = flight_.callbacks[i];
        for (Completion& fn : cb.second)
            fn(results + cb.first);
    });
    flight_.callbacks.clear();
    flight_.downloads.clear();
    flight_.active = false;
    const uint64_t t2 = now_ns();
    std::vector<Shard*> shards;
    {
        std::lock_guard<std::mutex> g(shardsMu_);
        for (auto& s : shards_)
            shards.push_back(s.get());
    }
    // each shard's released buffers go back to its own free lists
    pool().run(shards.size(), [&](size_t i) {
        Shard* s = shards[i];
        for (const DevBuf& b : s->flightFree) {
            const size_t cls = cap_class(b.cap);
            if (cls >= s->freeLists.size())
                s->freeLists.resize(cls + 1);
            s->freeLists[cls].push_back(b.ptr);
        }
        s->flightFree.clear();
        spill(*s);
    });
    const uint64_t t3 = now_ns();
    flushStats_.waitNs += t1 - t0;
    flushStats_.completeNs += t2 - t1;
    flushStats_.reclaimNs += t3 - t2;
    return true;
}

} // namespace sgpu
