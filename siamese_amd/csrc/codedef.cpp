// codedef.cpp -- cached LDPC pick sequences (see codedef.h).
#include "codedef.h"

#include <immintrin.h>

#include <cstdlib>

#include <memory>
#include <unordered_map>
#include <vector>

namespace sgpu {

namespace {

struct LdpcCache
{
    // (row, n) -> offsets; bounded so long single-stream runs (C3/C5, many
    // distinct n) do not grow it without limit
    std::unordered_map<uint64_t, std::unique_ptr<std::vector<uint32_t>>> map;
    size_t bytes = 0;
    std::vector<uint32_t> scratch;
    // direct-mapped by row in front of the map: the rows of one decode or
    // encode share n, so a lookup is one load instead of a hash-bucket walk
    // (cold in cache after the thread has driven other streams)
    struct Front
    {
        uint32_t row = ~0u, n = 0;
        const std::vector<uint32_t>* v = nullptr;
    } front[256];
};

void compute(unsigned row, unsigned n, std::vector<uint32_t>& out)
{
    const unsigned pairs = (n + kPairRate - 1) / kPairRate;
    out.resize(2 * (size_t)pairs);
    Pcg32 prng;
    prng.seed(row, n);
    const FastMod mod(n ? n : 1);
    for (unsigned i = 0; i < 2 * pairs; ++i)
        out[i] = mod(prng.next());
}

struct RowSelectTable
{
    RowSelect t[256];
    RowSelectTable()
    {
        for (unsigned row = 0; row < 256; ++row) {
            RowSelect& r = t[row];
            r.mask[0] = r.mask[1] = 0;
            for (unsigned lane = 0; lane < kLanes; ++lane) {
                const unsigned op = row_opcode(lane, row);
                r.opLo[lane] = (uint8_t)(op & 7);
                r.opHi[lane] = (uint8_t)(op >> 3);
                for (unsigned bit = 0; bit < 2 * kSums; ++bit)
                    if (op & (1u << bit))
                        r.mask[bit / kSums] |= 1u << (lane * kSums + bit % kSums);
            }
        }
    }
};

const RowSelectTable g_rowSelect;

} // namespace

const RowSelect& row_select(unsigned row) { return g_rowSelect.t[row & 255]; }

const uint32_t* ldpc_offsets(unsigned row, unsigned n, unsigned* count)
{
    // (on the heap: the library's TLS is initial-exec and must stay small)
    thread_local std::unique_ptr<LdpcCache> cachePtr;
    if (!cachePtr)
        cachePtr.reset(new LdpcCache);
    LdpcCache& cache = *cachePtr;
    LdpcCache::Front& f = cache.front[row & 255];
    if (f.row == row && f.n == n) {
        *count = (unsigned)f.v->size();
        return f.v->data();
    }
    const uint64_t key = ((uint64_t)row << 32) | n;
    auto it = cache.map.find(key);
    if (it == cache.map.end()) {
        constexpr size_t kMaxBytes = 64u << 20;
        const size_t need = 8 * (size_t)((n + kPairRate - 1) / kPairRate);
        if (need > kMaxBytes / 4) {
            compute(row, n, cache.scratch);
            *count = (unsigned)cache.scratch.size();
            return cache.scratch.data();
        }
        if (cache.bytes + need > kMaxBytes) {
            cache.map.clear();
            cache.bytes = 0;
            for (LdpcCache::Front& e : cache.front)
                e = LdpcCache::Front();
        }
        std::unique_ptr<std::vector<uint32_t>> v(new std::vector<uint32_t>);
        compute(row, n, *v);
        cache.bytes += need + 64;
        it = cache.map.emplace(key, std::move(v)).first;
    }
    f.row = row;
    f.n = n;
    f.v = it->second.get();
    *count = (unsigned)it->second->size();
    return it->second->data();
}

} // namespace sgpu
