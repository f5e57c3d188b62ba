// engine.cpp -- arena, programs and flush (see engine.h).
#include "engine.h"
#include "backend.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

namespace sgpu {

// ---------------------------------------------------------------------------
// Program

Program::~Program()
{
    if (eng_)
        eng_->forget(this);
}

void Program::touch()
{
    if (!dirty_) {
        dirty_ = true;
        eng_->register_dirty(this);
    }
}

Program::Segment& Program::seg()
{
    if (segs_.empty())
        segs_.emplace_back();
    return segs_.back();
}

void Program::lc_begin(uint64_t dst, uint32_t n, uint32_t valid, uint8_t mix)
{
    touch();
    Segment& s = seg();
    GfOp op;
    std::memset(&op, 0, sizeof(op));
    op.dst = dst;
    op.n = n;
    op.valid = valid < n ? valid : n;
    op.kind = OP_LINCOMB;
    op.mix = mix;
    op.termBegin = (uint32_t)s.terms.size();
    op.termCount = 0;
    s.ops.push_back(op);
    open_ = true;
}

void Program::lc_term(uint64_t src, uint32_t len, uint8_t coeff, uint8_t acc)
{
    Segment& s = seg();
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

void Program::lc_end()
{
    Segment& s = seg();
    GfOp& op = s.ops.back();
    open_ = false;
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
    Segment& s = seg();
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
    eng_->add_ingest(d, (uint32_t)-1);
}

uint32_t Program::solve(const std::vector<SolveRow>& rows, const std::vector<uint8_t>& coef,
                        uint32_t maxBytes)
{
    touch();
    seg(); // make sure the segment preceding this solve exists
    PendingSolve ps;
    std::memset(&ps.desc, 0, sizeof(ps.desc));
    ps.desc.m = (uint32_t)rows.size();
    ps.desc.maxBytes = maxBytes;
    ps.desc.result = eng_->reserve_results(ps.desc.m + 1);
    ps.rows = rows;
    ps.coef = coef;
    const uint32_t r = ps.desc.result;
    solves_.push_back(std::move(ps));
    segs_.emplace_back(); // ops after the solve go to the next segment
    return r;
}

// ---------------------------------------------------------------------------
// Engine: arena

Engine* Engine::global()
{
    static Engine e;
    return &e;
}

bool Engine::init(int device, const char** err)
{
    if (ready_)
        return true;
    if (!be_init(device, err))
        return false;
    ready_ = true;
    return true;
}

static uint32_t round_cap(uint32_t bytes)
{
    if (bytes < 64)
        return 64;
    if (bytes <= 4096)
        return (bytes + 63) & ~63u;
    if (bytes <= 131072)
        return (bytes + 1023) & ~1023u;
    return (bytes + 65535) & ~65535u;
}

std::vector<uint8_t*>* Engine::free_list(uint32_t cap)
{
    auto it = std::lower_bound(freeLists_.begin(), freeLists_.end(), cap,
                               [](const std::pair<uint32_t, std::vector<uint8_t*>>& a, uint32_t c) {
                                   return a.first < c;
                               });
    if (it == freeLists_.end() || it->first != cap)
        it = freeLists_.insert(it, std::make_pair(cap, std::vector<uint8_t*>()));
    return &it->second;
}

DevBuf Engine::alloc(uint32_t bytes)
{
    DevBuf b;
    const uint32_t cap = round_cap(bytes);
    std::vector<uint8_t*>* fl = free_list(cap);
    if (!fl->empty()) {
        b.ptr = fl->back();
        fl->pop_back();
        b.cap = cap;
        inUse_ += cap;
        return b;
    }
    const size_t kChunk = 64u << 20;
    if (cap > kChunk / 4) {
        b.ptr = (uint8_t*)be_dev_alloc(cap);
        if (!b.ptr)
            return DevBuf();
        b.cap = cap;
        inUse_ += cap;
        return b;
    }
    if (chunks_.empty() || chunks_.back().used + cap > chunks_.back().size) {
        uint8_t* base = (uint8_t*)be_dev_alloc(kChunk);
        if (!base)
            return DevBuf();
        chunks_.push_back(Chunk{base, kChunk, 0});
    }
    Chunk& c = chunks_.back();
    b.ptr = c.base + c.used;
    b.cap = cap;
    c.used += cap;
    inUse_ += cap;
    return b;
}

void Engine::release(DevBuf& b)
{
    if (b.ptr) {
        pendingFree_.push_back(b);
        inUse_ -= b.cap;
    }
    b = DevBuf();
}

void Engine::forget(Program* p)
{
    auto it = std::find(dirty_.begin(), dirty_.end(), p);
    if (it != dirty_.end())
        dirty_.erase(it);
}

void Engine::download(void* hostDst, uint64_t devSrc, uint32_t bytes)
{
    if (bytes)
        downloads_.push_back(Download{hostDst, devSrc, bytes});
}

void Engine::on_complete(std::function<void(const uint32_t*)> fn)
{
    callbacks_.push_back(std::move(fn));
}

void Engine::stage_host_ingest(const DevBuf& dst, const void* data, uint32_t bytes,
                               const uint8_t* hdr, uint32_t hdrLen)
{
    // Stage hdr || data contiguously so the device copy is aligned.
    const size_t off = (hostStage_.size() + 15) & ~(size_t)15;
    hostStage_.resize(off + hdrLen + bytes);
    std::memcpy(hostStage_.data() + off, hdr, hdrLen);
    std::memcpy(hostStage_.data() + off + hdrLen, data, bytes);
    IngestDesc d;
    std::memset(&d, 0, sizeof(d));
    d.dst = dst.addr();
    d.src = 0;
    d.bytes = hdrLen + bytes;
    d.hdrLen = 0;
    add_ingest(d, (uint32_t)off);
}

void Engine::add_ingest(const IngestDesc& d, uint32_t hostStageOffset)
{
    IngestRec r;
    r.d = d;
    r.hostOffset = hostStageOffset == (uint32_t)-1 ? -1 : (int64_t)hostStageOffset;
    ingest_.push_back(r);
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

namespace {

inline size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

struct Phase
{
    enum Kind { EXEC, SOLVE } kind;
    size_t itemBegin, itemCount;    // exec items or solve items
    size_t solveBegin, solveCount;  // solve descs (SOLVE)
};

} // namespace

void Engine::flush()
{
    if (flight_.active)
        sync();
    if (!pending() && callbacks_.empty() && pendingFree_.empty())
        return;

    // ---- gather host-side arrays --------------------------------------
    std::vector<IngestDesc> ingDescs;
    std::vector<IngestItem> ingItems;
    ingDescs.reserve(ingest_.size());
    for (const IngestRec& r : ingest_) {
        const uint32_t idx = (uint32_t)ingDescs.size();
        ingDescs.push_back(r.d);
        const uint32_t total = r.d.hdrLen + r.d.bytes;
        for (uint32_t t = 0; t < total; t += kTileBytes)
            ingItems.push_back(IngestItem{idx, t});
    }

    std::vector<GfOp> ops;
    std::vector<GfTerm> terms;
    std::vector<ExecItem> items;
    std::vector<SolveDesc> sdescs;
    std::vector<SolveRow> srows;
    std::vector<uint8_t> coef;
    std::vector<SolveItem> sitems;
    std::vector<Phase> phases;

    for (int group = 0; group < 2; ++group) {
        size_t maxSegs = 0;
        for (Program* p : dirty_)
            if (p->group_ == group)
                maxSegs = std::max(maxSegs, p->segs_.size());
        for (size_t k = 0; k < maxSegs; ++k) {
            Phase ex{Phase::EXEC, items.size(), 0, 0, 0};
            for (Program* p : dirty_) {
                if (p->group_ != group || k >= p->segs_.size())
                    continue;
                Program::Segment& s = p->segs_[k];
                if (s.ops.empty())
                    continue;
                const uint32_t opBase = (uint32_t)ops.size();
                const uint32_t termBase = (uint32_t)terms.size();
                for (GfOp op : s.ops) {
                    if (op.kind == OP_LINCOMB)
                        op.termBegin += termBase;
                    ops.push_back(op);
                }
                terms.insert(terms.end(), s.terms.begin(), s.terms.end());
                for (uint32_t t = 0; t < s.maxExtent; t += kTileBytes)
                    items.push_back(ExecItem{opBase, (uint32_t)s.ops.size(), t, 0});
            }
            ex.itemCount = items.size() - ex.itemBegin;
            if (ex.itemCount)
                phases.push_back(ex);

            Phase sv{Phase::SOLVE, sitems.size(), 0, sdescs.size(), 0};
            for (Program* p : dirty_) {
                if (p->group_ != group || k >= p->solves_.size())
                    continue;
                Program::PendingSolve& ps = p->solves_[k];
                SolveDesc d = ps.desc;
                d.rowBegin = (uint32_t)srows.size();
                d.coefOffset = coef.size();
                srows.insert(srows.end(), ps.rows.begin(), ps.rows.end());
                coef.insert(coef.end(), ps.coef.begin(), ps.coef.end());
                const uint32_t sidx = (uint32_t)sdescs.size();
                sdescs.push_back(d);
                for (uint32_t t = 0; t < d.maxBytes; t += kTileBytes)
                    sitems.push_back(SolveItem{sidx, t});
            }
            sv.itemCount = sitems.size() - sv.itemBegin;
            sv.solveCount = sdescs.size() - sv.solveBegin;
            if (sv.solveCount)
                phases.push_back(sv);
        }
    }

    // ---- lay out the single upload --------------------------------------
    size_t off = 0;
    const size_t oStage = off;
    off = align16(off + hostStage_.size());
    const size_t oIngD = off;
    off = align16(off + ingDescs.size() * sizeof(IngestDesc));
    const size_t oIngI = off;
    off = align16(off + ingItems.size() * sizeof(IngestItem));
    const size_t oOps = off;
    off = align16(off + ops.size() * sizeof(GfOp));
    const size_t oTerms = off;
    off = align16(off + terms.size() * sizeof(GfTerm));
    const size_t oItems = off;
    off = align16(off + items.size() * sizeof(ExecItem));
    const size_t oSD = off;
    off = align16(off + sdescs.size() * sizeof(SolveDesc));
    const size_t oSR = off;
    off = align16(off + srows.size() * sizeof(SolveRow));
    const size_t oCoef = off;
    off = align16(off + coef.size());
    const size_t oSI = off;
    off = align16(off + sitems.size() * sizeof(SolveItem));
    const size_t upBytes = off;

    if (upBytes)
        ensure_up(upBytes);
    for (size_t i = 0; i < ingest_.size(); ++i)
        if (ingest_[i].hostOffset >= 0)
            ingDescs[i].src = (uint64_t)(uintptr_t)(upDev_ + oStage + ingest_[i].hostOffset);

    auto put = [&](size_t o, const void* src, size_t n) {
        if (n)
            std::memcpy(upHost_ + o, src, n);
    };
    put(oStage, hostStage_.data(), hostStage_.size());
    put(oIngD, ingDescs.data(), ingDescs.size() * sizeof(IngestDesc));
    put(oIngI, ingItems.data(), ingItems.size() * sizeof(IngestItem));
    put(oOps, ops.data(), ops.size() * sizeof(GfOp));
    put(oTerms, terms.data(), terms.size() * sizeof(GfTerm));
    put(oItems, items.data(), items.size() * sizeof(ExecItem));
    put(oSD, sdescs.data(), sdescs.size() * sizeof(SolveDesc));
    put(oSR, srows.data(), srows.size() * sizeof(SolveRow));
    put(oCoef, coef.data(), coef.size());
    put(oSI, sitems.data(), sitems.size() * sizeof(SolveItem));

    // download area: results first, then each requested range
    size_t dOff = align16((size_t)resultWords_ * 4);
    std::vector<Download> dls = downloads_;
    std::vector<size_t> dlOff;
    for (const Download& d : dls) {
        dlOff.push_back(dOff);
        dOff = align16(dOff + d.bytes);
    }
    if (dOff)
        ensure_down(dOff);

    // ---- launch ----------------------------------------------------------
    if (upBytes)
        be_h2d(upDev_, upHost_, upBytes);
    if (!ingItems.empty())
        be_launch_ingest((const IngestDesc*)(upDev_ + oIngD), (const IngestItem*)(upDev_ + oIngI),
                         (uint32_t)ingItems.size());
    uint32_t* resultsDev = (uint32_t*)downDev_;
    for (const Phase& ph : phases) {
        if (ph.kind == Phase::EXEC) {
            be_launch_exec((const GfOp*)(upDev_ + oOps), (const GfTerm*)(upDev_ + oTerms),
                           (const ExecItem*)(upDev_ + oItems) + ph.itemBegin, (uint32_t)ph.itemCount);
        } else {
            const SolveDesc* sd = (const SolveDesc*)(upDev_ + oSD) + ph.solveBegin;
            be_launch_solve_prefix(sd, (const SolveRow*)(upDev_ + oSR), upDev_ + oCoef, resultsDev,
                                   (uint32_t)ph.solveCount);
            // solve items index solves globally; pass the global desc base
            be_launch_solve_main((const SolveDesc*)(upDev_ + oSD), (const SolveRow*)(upDev_ + oSR),
                                 upDev_ + oCoef, resultsDev,
                                 (const SolveItem*)(upDev_ + oSI) + ph.itemBegin,
                                 (uint32_t)ph.itemCount);
        }
    }
    if (resultWords_)
        be_d2h(downHost_, resultsDev, (size_t)resultWords_ * 4);
    for (size_t i = 0; i < dls.size(); ++i)
        be_d2h(downHost_ + dlOff[i], (const void*)(uintptr_t)dls[i].dev, dls[i].bytes);

    // ---- bookkeeping -----------------------------------------------------
    stats.flushes++;
    stats.launches += phases.size() + (ingItems.empty() ? 0 : 1);
    stats.ops += ops.size();
    stats.terms += terms.size();
    stats.solves += sdescs.size();
    stats.ingests += ingDescs.size();
    stats.uploadBytes += upBytes;

    flight_.downloads.clear();
    for (size_t i = 0; i < dls.size(); ++i)
        flight_.downloads.push_back(Download{dls[i].host, (uint64_t)dlOff[i], dls[i].bytes});
    flight_.callbacks.swap(callbacks_);
    callbacks_.clear();
    flight_.resultWords = resultWords_;
    flight_.active = true;
    // Buffers released before this flush may be reused once it completes.
    flightFree_.swap(pendingFree_);
    pendingFree_.clear();

    for (Program* p : dirty_) {
        p->segs_.clear();
        p->solves_.clear();
        p->dirty_ = false;
    }
    dirty_.clear();
    ingest_.clear();
    hostStage_.clear();
    downloads_.clear();
    resultWords_ = 0;
}

bool Engine::gather(unsigned count, const void* const* srcs, const unsigned* bytes, void* hostOut)
{
    if (flight_.active)
        sync();
    if (count == 0)
        return true;
    std::vector<IngestDesc> descs(count);
    std::vector<IngestItem> items;
    size_t total = 0;
    for (unsigned i = 0; i < count; ++i) {
        std::memset(&descs[i], 0, sizeof(IngestDesc));
        descs[i].src = (uint64_t)(uintptr_t)srcs[i];
        descs[i].bytes = bytes[i];
        descs[i].dst = total; // offset for now
        for (uint32_t t = 0; t < bytes[i]; t += kTileBytes)
            items.push_back(IngestItem{i, t});
        total = align16(total + bytes[i]);
    }
    const size_t dBytes = count * sizeof(IngestDesc);
    const size_t upBytes = align16(dBytes) + items.size() * sizeof(IngestItem);
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
    std::memcpy(gUpHost_, descs.data(), dBytes);
    std::memcpy(gUpHost_ + align16(dBytes), items.data(), items.size() * sizeof(IngestItem));
    be_h2d(gUpDev_, gUpHost_, upBytes);
    if (!items.empty())
        be_launch_ingest((const IngestDesc*)gUpDev_, (const IngestItem*)(gUpDev_ + align16(dBytes)),
                         (uint32_t)items.size());
    be_d2h(gHost_, gDev_, total);
    const bool ok = be_sync();
    uint8_t* out = (uint8_t*)hostOut;
    size_t off = 0;
    for (unsigned i = 0; i < count; ++i) {
        std::memcpy(out, gHost_ + off, bytes[i]);
        out += bytes[i];
        off = align16(off + bytes[i]);
    }
    return ok;
}

bool Engine::sync()
{
    if (!flight_.active)
        return true;
    const bool ok = be_sync();
    for (const Download& d : flight_.downloads)
        std::memcpy(d.host, downHost_ + d.dev, d.bytes);
    const uint32_t* results = (const uint32_t*)downHost_;
    for (auto& fn : flight_.callbacks)
        fn(results);
    flight_.callbacks.clear();
    flight_.downloads.clear();
    flight_.active = false;
    for (DevBuf& b : flightFree_) {
        free_list(b.cap)->push_back(b.ptr);
    }
    flightFree_.clear();
    return ok;
}

} // namespace sgpu
