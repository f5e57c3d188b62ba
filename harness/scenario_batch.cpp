// harness/scenario_batch.cpp -- lock-step batched driver over the
// device-resident API (include/siamese_gpu.h) of libsiamese_amd.
//
// Every stream runs the same Stream<> state machine as the per-call driver,
// so each stream issues the identical call sequence; only the interleaving
// across streams differs.  A round advances every live stream until it
// yields (after a successful decode, whose recovered lengths the device
// resolves at the flush), then one sgpu_flush() executes the round's device
// work for all streams in a few kernel launches.
//
// Originals are staged in HBM once before timing starts ("device-resident").
//
// Exported (ctypes):
//   int scenario_run_batch(const char* lib, const ScenarioConfig* cfg,
//                          StreamResult* results, const BatchOptions* opt,
//                          BatchReport* report)
#include "scenario.h"
#include "../include/siamese_gpu.h"
#include "../siamese_amd/csrc/pool.h"

#include <dlfcn.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <malloc.h>
#include <memory>
#include <mutex>

extern "C" {

struct BatchOptions
{
    uint32_t steps;    ///< timed repetitions of the whole workload
    uint32_t warmup;   ///< untimed repetitions before timing
    uint32_t verify;   ///< check every recovered packet's bytes (first run only)
    int32_t device;    ///< HIP device (-1 = current)
    uint32_t threads;  ///< host threads driving streams (0 = default)
    uint32_t groups;   ///< stream groups alternating host work and device work (0 = 1)
    uint32_t e2e;      ///< originals start in pinned host memory (H2D each step) and every
                       ///< recovery packet and recovered original is copied back (D2H)
    uint32_t digest;   ///< keep event logs and digests on unverified runs too
    uint32_t defer;    ///< 0: a stream yields after each decode and waits for its
                       ///< submission (sgpu_decode / sgpu_decoder_get);
                       ///< k > 0: deferred outputs (sgpu_decode_deferred /
                       ///< sgpu_decoder_get_deferred), a stream yields after
                       ///< every k-th decode and a job is driven on with up to
                       ///< two of its submissions in flight
    uint32_t frames;   ///< with e2e: packets travel as framed datagrams (siamese_gpu.h):
                       ///< originals staged as frames and handed to the decoders by
                       ///< sgpu_frames_recv, recovery packets copied back framed by
                       ///< sgpu_frames_send and parsed on landing
    uint32_t no_timing; ///< timed steps without the per-launch device timing events
    uint32_t device_ge; ///< defer 0: decodes by sgpu_decode_device (recovery matrix generated and
                        ///< eliminated on the device; a decode then takes two submissions)
    uint32_t unique;    ///< count the executor launches' compulsory bytes (sgpu_measure_unique)
                        ///< during the run (a measurement run: it costs assembly time)
                        ///< (device_ms / exec_ms read 0): the events order every launch
                        ///< behind a timestamp, tens of microseconds a flush on the
                        ///< latency-bound single-stream legs
};

struct BatchReport
{
    double seconds;        ///< wall time of the timed steps (total)
    double device_ms;      ///< device time of all launches in the timed steps
    double exec_ms;        ///< device time of the executor launches only
    double setup_seconds;  ///< payload generation + staging (untimed)
    uint64_t rounds;       ///< rounds (flushes) in the timed steps
    uint64_t engine[21];   ///< engine counters over the timed steps (see sgpu_engine_stats_ex),
                           ///< then the arena growth (sgpu_arena_bytes)
    uint64_t checked;      ///< packets whose bytes were verified
    uint64_t mismatches;   ///< verification failures
    /// wall time of the timed steps split by phase: codec create, stream
    /// stepping (host control plane), sgpu_flush (assembly + upload + device
    /// + completion), token resolution, finish + free
    double phase_seconds[5];
    uint64_t payload_bytes;   ///< payload bytes of the originals added in the timed steps (all steps)
    double kernel_ms[5];      ///< device time by kernel class (sgpu_timing_kernels)
};

} // extern "C"

namespace {

constexpr int kEngineStats = 20;
using Clock = std::chrono::steady_clock;

struct Api
{
    int (*init)(int);
    SgpuEncoder (*encoder_create)(void);
    void (*encoder_free)(SgpuEncoder);
    SiameseResult (*encoder_add)(SgpuEncoder, const void*, unsigned, unsigned*);
    SiameseResult (*encoder_remove_before)(SgpuEncoder, unsigned);
    SiameseResult (*encode)(SgpuEncoder, SgpuRecoveryPacket*);
    SiameseResult (*encode_range)(SgpuEncoder, SgpuRecoveryPacket*, unsigned, unsigned*);
    SgpuDecoder (*decoder_create)(void);
    void (*decoder_free)(SgpuDecoder);
    SiameseResult (*decoder_add_original)(SgpuDecoder, unsigned, const void*, unsigned);
    SiameseResult (*decoder_add_recovery)(SgpuDecoder, const SgpuRecoveryPacket*);
    SiameseResult (*decoder_is_ready)(SgpuDecoder);
    SiameseResult (*decode)(SgpuDecoder, SiameseOriginalPacket**, unsigned*);
    SiameseResult (*decoder_get)(SgpuDecoder, SiameseOriginalPacket*);
    SiameseResult (*decode_deferred)(SgpuDecoder, SiameseOriginalPacket*, unsigned, unsigned*);
    SiameseResult (*decoder_get_deferred)(SgpuDecoder, SiameseOriginalPacket*);
    SiameseResult (*encoder_add_range)(SgpuEncoder, const void*, size_t, const unsigned*, unsigned, unsigned,
                                       unsigned*, unsigned*);
    SiameseResult (*decoder_add_original_range)(SgpuDecoder, unsigned, const void*, size_t, const unsigned*,
                                                unsigned, unsigned, SiameseResult*, unsigned*);
    SiameseResult (*decoder_get_range)(SgpuDecoder, unsigned, unsigned, SiameseOriginalPacket*, unsigned*);
    SiameseResult (*decode_device)(SgpuDecoder, SiameseOriginalPacket**, unsigned*);
    int (*flush)(void);
    int (*submit)(void);
    long long (*enqueue)(void);
    int (*wait)(long long);
    int (*query)(long long);
    void (*parallel_for)(unsigned, void (*)(void*, unsigned), void*);
    void* (*device_alloc)(size_t);
    void (*device_free)(void*);
    void* (*host_alloc)(size_t);
    void (*host_free)(void*);
    int (*h2d)(void*, const void*, size_t);
    int (*gather)(unsigned, const void* const*, const unsigned*, void*);
    int (*h2d_async)(void*, const void*, size_t);
    int (*gather_completed)(unsigned, const void* const*, const unsigned*, void*);
    long long (*gather_async)(unsigned, const void* const*, const unsigned*, void*);
    unsigned (*frame_header_bytes)(unsigned, unsigned);
    unsigned (*frame_write_header)(unsigned, unsigned, unsigned, unsigned, void*);
    SiameseResult (*frames_parse)(const void*, size_t, SgpuFrame*, unsigned, unsigned*);
    SiameseResult (*frames_recv)(const SgpuDecoder*, unsigned, const void*, const void*, size_t, SiameseResult*,
                                 unsigned, unsigned*);
    long long (*frames_send)(unsigned, const SgpuRecoveryPacket*, const unsigned*, void*, size_t, size_t*);
    int (*gather_wait)(long long);
    void (*timing)(int, int, double*, double*);
    void (*engine_stats)(uint64_t*);
    void (*engine_stats_ex)(uint64_t*, unsigned);
    void (*measure_unique)(int);
    void (*timing_kernels)(double*, unsigned);
    uint64_t (*arena_bytes)(void);
    int (*arena_reserve)(size_t);
};

template <class F>
bool bind(void* h, F& fn, const char* name)
{
    fn = reinterpret_cast<F>(dlsym(h, name));
    if (!fn)
        std::fprintf(stderr, "scenario_batch: missing symbol %s\n", name);
    return fn != nullptr;
}

// (range calls are optional: a library without them -- an older build in
// an A/B -- gets loops of the single calls, the same call results)
template <class F>
bool bind_optional(void* h, F& fn, const char* name)
{
    fn = reinterpret_cast<F>(dlsym(h, name));
    return true;
}

bool load_api(const char* path, Api& a)
{
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        std::fprintf(stderr, "scenario_batch: dlopen(%s) failed: %s\n", path, dlerror());
        return false;
    }
    return bind(h, a.init, "sgpu_init") && bind(h, a.encoder_create, "sgpu_encoder_create") &&
           bind(h, a.encoder_free, "sgpu_encoder_free") && bind(h, a.encoder_add, "sgpu_encoder_add") &&
           bind(h, a.encoder_remove_before, "sgpu_encoder_remove_before") &&
           bind(h, a.encode, "sgpu_encode") && bind(h, a.decoder_create, "sgpu_decoder_create") &&
           bind(h, a.decoder_free, "sgpu_decoder_free") &&
           bind(h, a.decoder_add_original, "sgpu_decoder_add_original") &&
           bind(h, a.decoder_add_recovery, "sgpu_decoder_add_recovery") &&
           bind(h, a.decoder_is_ready, "sgpu_decoder_is_ready") && bind(h, a.decode, "sgpu_decode") &&
           bind(h, a.decoder_get, "sgpu_decoder_get") && bind(h, a.decode_deferred, "sgpu_decode_deferred") &&
           bind(h, a.decoder_get_deferred, "sgpu_decoder_get_deferred") &&
           bind(h, a.flush, "sgpu_flush") && bind(h, a.submit, "sgpu_submit") &&
           bind(h, a.enqueue, "sgpu_enqueue") && bind(h, a.wait, "sgpu_wait") &&
           bind(h, a.query, "sgpu_query") &&
           bind(h, a.parallel_for, "sgpu_parallel_for") &&
           bind(h, a.device_alloc, "sgpu_device_alloc") && bind(h, a.device_free, "sgpu_device_free") &&
           bind(h, a.host_alloc, "sgpu_host_alloc") && bind(h, a.host_free, "sgpu_host_free") &&
           bind(h, a.h2d, "sgpu_h2d") && bind(h, a.gather, "sgpu_gather") &&
           bind(h, a.h2d_async, "sgpu_h2d_async") && bind(h, a.gather_completed, "sgpu_gather_completed") &&
           bind(h, a.gather_async, "sgpu_gather_async") && bind(h, a.gather_wait, "sgpu_gather_wait") &&
           bind(h, a.frame_header_bytes, "sgpu_frame_header_bytes") &&
           bind(h, a.frame_write_header, "sgpu_frame_write_header") && bind(h, a.frames_parse, "sgpu_frames_parse") &&
           bind(h, a.frames_recv, "sgpu_frames_recv") && bind(h, a.frames_send, "sgpu_frames_send") &&
           bind(h, a.timing, "sgpu_timing") && bind(h, a.engine_stats, "sgpu_engine_stats") &&
           bind(h, a.arena_bytes, "sgpu_arena_bytes") && bind(h, a.arena_reserve, "sgpu_arena_reserve") &&
           bind_optional(h, a.encoder_add_range, "sgpu_encoder_add_range") &&
           bind_optional(h, a.decoder_add_original_range, "sgpu_decoder_add_original_range") &&
           bind_optional(h, a.decoder_get_range, "sgpu_decoder_get_range") &&
           bind_optional(h, a.engine_stats_ex, "sgpu_engine_stats_ex") &&
           bind_optional(h, a.measure_unique, "sgpu_measure_unique") &&
           bind_optional(h, a.encode_range, "sgpu_encode_range") &&
           bind_optional(h, a.timing_kernels, "sgpu_timing_kernels") &&
           bind_optional(h, a.decode_device, "sgpu_decode_device");
}

// SCENARIO_BATCH_CALLS=1: time every codec call by kind (TSC ticks, summed
// per thread without shared atomics so the counting does not perturb a
// multithreaded run) and print the totals after each run (diagnostic)
enum CallKind { kEncAdd, kEncode, kDecAddOrig, kDecAddRec, kIsReady, kDecode, kDecGet, kRemove, kCreate, kFree,
                kCallKinds };
const char* const kCallNames[kCallKinds] = {"enc_add", "encode", "dec_add_orig", "dec_add_rec", "is_ready",
                                            "decode", "dec_get", "remove", "create", "free"};
const bool kCallTiming = std::getenv("SCENARIO_BATCH_CALLS") != nullptr;
struct CallCounts
{
    uint64_t v[kCallKinds][3] = {};   // calls, ticks, items
    uint64_t busy = 0;                // ticks inside for_streams tasks
};
std::atomic<uint64_t> g_fjWall{0}, g_fjCount{0};   // for_streams: wall ticks, fork-joins
std::mutex g_callsMu;
std::vector<CallCounts*> g_callCounts;   // one per thread that timed a call (never freed)
CallCounts& call_counts()
{
    thread_local CallCounts* c = nullptr;
    if (!c) {
        c = new CallCounts;
        std::lock_guard<std::mutex> g(g_callsMu);
        g_callCounts.push_back(c);
    }
    return *c;
}

struct CallTimer
{
    CallKind k;
    uint64_t items;
    uint64_t t0 = 0;
    explicit CallTimer(CallKind kind, uint64_t n = 1) : k(kind), items(n)
    {
        if (kCallTiming)
            t0 = __builtin_ia32_rdtsc();
    }
    ~CallTimer()
    {
        if (!kCallTiming)
            return;
        CallCounts& c = call_counts();
        c.v[k][0] += 1;
        c.v[k][1] += __builtin_ia32_rdtsc() - t0;
        c.v[k][2] += items;
    }
};

void print_calls()
{
    if (!kCallTiming)
        return;
    // TSC rate from a short wall-clock window
    const auto w0 = Clock::now();
    const uint64_t c0 = __builtin_ia32_rdtsc();
    while (Clock::now() - w0 < std::chrono::milliseconds(20)) {
    }
    const double ticksPerNs =
        (double)(__builtin_ia32_rdtsc() - c0) / (double)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - w0).count();
    std::lock_guard<std::mutex> g(g_callsMu);
    {
        uint64_t busy = 0;
        unsigned threads = 0;
        for (CallCounts* cc : g_callCounts) {
            busy += cc->busy;
            threads += cc->busy ? 1 : 0;
            cc->busy = 0;
        }
        const uint64_t wall = g_fjWall.exchange(0), n = g_fjCount.exchange(0);
        if (wall)
            std::fprintf(stderr, "batch fork-joins %llu: wall %.1f us, busy %.1f us on %u threads, "
                         "busy/(wall*threads) %.3f\n", (unsigned long long)n, wall / ticksPerNs / 1e3,
                         busy / ticksPerNs / 1e3, threads, threads ? (double)busy / ((double)wall * threads) : 0.0);
    }
    for (unsigned k = 0; k < kCallKinds; ++k) {
        uint64_t c = 0, t = 0, it = 0;
        for (CallCounts* cc : g_callCounts) {
            c += cc->v[k][0];
            t += cc->v[k][1];
            it += cc->v[k][2];
            cc->v[k][0] = cc->v[k][1] = cc->v[k][2] = 0;
        }
        const double ns = (double)t / ticksPerNs;
        if (c)
            std::fprintf(stderr, "batch %-13s %9llu calls %9llu items %10.1f us  %8.3f us/item\n", kCallNames[k],
                         (unsigned long long)c, (unsigned long long)it, ns / 1e3, ns / 1e3 / (double)it);
    }
}

struct Rec
{
    unsigned bytes = 0;
    SgpuRecoveryPacket pkt{};
};

struct Pkt
{
    unsigned num = 0, bytes = 0;
    const unsigned char* data = nullptr;          // device pointer (get)
    const SiameseOriginalPacket* entry = nullptr; // decode output entry (resolved at flush)
};

// A token whose value needs device results, resolved once the submission
// that closed the round it was made in has completed.
struct Request
{
    std::vector<uint64_t>* log;
    size_t pos;
    const void* dev;
    unsigned bytes;
    unsigned id;     // payload id to verify against (packets only)
    bool isPacket;
    bool* ok;
    const SiameseOriginalPacket* entry = nullptr;   // deferred output: dev/bytes read at resolution
    unsigned* inFlight = nullptr;                   // its codec's count of unresolved requests
};

struct Shared
{
    const Api* api;
    const ScenarioConfig* cfg;
    uint8_t* payload;        // all originals, device-resident (indexed by global payload id)
    uint8_t* payload2 = nullptr;   // e2e: the second device copy (steps alternate, see run_pipeline)
    size_t stride;
    bool hashData;
    bool verify;
    bool e2e = false;         // packets start and end in host memory (timed copies)
    uint8_t* hostPayload = nullptr;   // pinned host copy of every original (e2e)
    uint8_t* devBase = nullptr;       // its device-resident counterparts
    uint8_t* devBase2 = nullptr;
    size_t payloadBytes = 0;
    // framed datagrams (BatchOptions::frames, with e2e): every original as a
    // frame in a pinned ring at a fixed stride, and its two device copies
    bool frames = false;
    uint8_t* frameHost = nullptr;
    uint8_t* frameDev = nullptr;
    uint8_t* frameDev2 = nullptr;
    size_t fstride = 0, frameBytes = 0;
    uint64_t idBase = 0;       // global payload id of the session's first original
    // gathers in flight (oldest first) and their pinned landing buffers
    struct Landing
    {
        uint8_t* buf = nullptr;
        size_t cap = 0;
    };
    struct Gather
    {
        long long ticket;
        Landing land;
        std::vector<Request> reqs;   // kept only when the bytes are checked or hashed
        bool framed = false;         // landed as frames (sgpu_frames_send)
        size_t bytes = 0;            // framed: the frame stream's length
    };
    std::deque<Gather> gathers;
    std::vector<Landing> landings;    // free ones
    uint64_t checked = 0, mismatches = 0;
    std::unique_ptr<sgpu::WorkerPool> pool;
    unsigned groups = 1;
    bool digest = true;   // per-stream digests (event logs) also on unverified runs
    unsigned defer = 0;   // BatchOptions::defer
    bool deviceGe = false;   // BatchOptions::device_ge (and the library has it)
};

struct BatchCodec
{
    Shared* sh;
    const uint8_t* payload = nullptr;   // the step's device copy of the originals
    const SgpuDecoder* decTable = nullptr;   // frames: the job's decoders by flow (stream index)
    unsigned flow = 0;                       // frames: this stream's flow id
    SgpuEncoder enc = nullptr;
    SgpuDecoder dec = nullptr;
    std::vector<uint64_t>* log = nullptr;
    std::vector<Request> cur;           // tokens made in the current round
    unsigned inFlight = 0;              // tokens made in rounds not yet resolved
    unsigned decodes = 0;               // decodes since the last yield (deferred mode)
    // deferred outputs: caller-owned entries the library fills at completion
    // (stable addresses, kept until the job retires)
    std::vector<std::unique_ptr<SiameseOriginalPacket[]>> slabs;
    unsigned slabUsed = kSlab;
    static constexpr unsigned kSlab = 1024;
    SiameseOriginalPacket* entries(unsigned n)
    {
        if (slabUsed + n > kSlab) {
            slabs.emplace_back(new SiameseOriginalPacket[kSlab]);
            slabUsed = 0;
        }
        SiameseOriginalPacket* e = slabs.back().get() + slabUsed;
        slabUsed += n;
        return e;
    }

    unsigned payload_bytes(unsigned id) const
    {
        return sh->cfg->payload_bytes ? sh->cfg->payload_bytes : scen::variable_bytes(id);
    }
    const void* dev_payload(unsigned id) const
    {
        if (sh->frames)   // (the payload after the frame's header)
            return payload + (id - sh->idBase) * sh->fstride +
                   sh->api->frame_header_bytes(SGPU_FRAME_ORIGINAL, payload_bytes(id));
        return payload + (size_t)id * sh->stride;
    }

    bool needs_host_payload() const { return false; }
    int enc_add(unsigned id, const uint8_t*, unsigned bytes, unsigned* num)
    {
        CallTimer ct(kEncAdd);
        return sh->api->encoder_add(enc, dev_payload(id), bytes, num);
    }
    // encode_hint: packets made ahead by one sgpu_encode_range, handed out
    // by the encode() calls that follow (the same packets, in order)
    std::vector<SgpuRecoveryPacket> ahead;
    unsigned aheadNext = 0;
    int aheadFail = 0;   // the range's result when it stopped early (returned after the packets)
    void encode_hint(unsigned n)
    {
        if (n < 2 || !sh->api->encode_range || aheadNext < ahead.size() || aheadFail)
            return;
        ahead.resize(n);
        unsigned made = 0;
        CallTimer ct(kEncode, n);
        const int r = sh->api->encode_range(enc, ahead.data(), n, &made);
        ahead.resize(made);
        aheadNext = 0;
        aheadFail = r;
    }
    int encode(Rec* r)
    {
        if (aheadNext < ahead.size()) {
            r->pkt = ahead[aheadNext++];
            r->bytes = r->pkt.DataBytes;
            return 0;
        }
        if (aheadFail) {
            const int res = aheadFail;
            aheadFail = 0;
            r->pkt.DataBytes = 0;
            r->bytes = 0;
            return res;
        }
        CallTimer ct(kEncode);
        const int res = sh->api->encode(enc, &r->pkt);
        r->bytes = r->pkt.DataBytes;
        return res;
    }
    int dec_add_original(unsigned id, unsigned num, const uint8_t*, unsigned bytes)
    {
        if (sh->frames) {
            // the datagram as it arrives: its frame in the pinned ring (the
            // header rewritten with the packet number the encoder gave it),
            // whose device copy the job staged; parsed and routed by the library
            const size_t slot = (id - sh->idBase) * sh->fstride;
            uint8_t* f = sh->frameHost + slot;
            const unsigned h = sh->api->frame_write_header(SGPU_FRAME_ORIGINAL, flow, num, bytes, f);
            SiameseResult r = Siamese_InvalidInput;
            unsigned n = 0;
            if (h == 0)
                return Siamese_InvalidInput;
            // (the call's status is the frame's result; n says whether it was taken)
            (void)sh->api->frames_recv(decTable, sh->cfg->streams, f, payload + slot, h + bytes, &r, 1, &n);
            return n == 1 ? r : Siamese_InvalidInput;
        }
        CallTimer ct(kDecAddOrig);
        return sh->api->decoder_add_original(dec, num, dev_payload(id), bytes);
    }
    int dec_add_recovery(const Rec& r)
    {
        CallTimer ct(kDecAddRec);
        return sh->api->decoder_add_recovery(dec, &r.pkt);
    }
    int is_ready()
    {
        CallTimer ct(kIsReady);
        return sh->api->decoder_is_ready(dec);
    }
    int decode(std::vector<Pkt>* out)
    {
        SiameseOriginalPacket* p = nullptr;
        unsigned n = 0;
        int r;
        CallTimer ct(kDecode);
        if (sh->defer) {
            // (capacity: a solve's 255 packets or what single recoveries hold;
            // unused entries are handed back)
            constexpr unsigned kCap = 255;
            p = entries(kCap);
            r = sh->api->decode_deferred(dec, p, kCap, &n);
            slabUsed -= kCap - (r == 0 ? n : 0);
        } else if (sh->deviceGe) {
            r = sh->api->decode_device(dec, &p, &n);
        } else {
            r = sh->api->decode(dec, &p, &n);
        }
        if (r == 0)
            for (unsigned i = 0; i < n; ++i) {
                Pkt k;
                k.num = p[i].PacketNum;
                k.entry = &p[i];
                out->push_back(k);
            }
        return r;
    }
    int dec_get(unsigned num, Pkt* out)
    {
        if (sh->defer) {
            SiameseOriginalPacket* e = entries(1);
            e->PacketNum = num;
            e->Data = nullptr;
            e->DataBytes = 0;
            const int r = sh->api->decoder_get_deferred(dec, e);
            if (r != 0)
                --slabUsed;
            out->num = num;
            out->entry = r == 0 ? e : nullptr;
            return r;
        }
        SiameseOriginalPacket p;
        p.PacketNum = num;
        p.Data = nullptr;
        p.DataBytes = 0;
        CallTimer ct(kDecGet);
        const int r = sh->api->decoder_get(dec, &p);
        out->num = num;
        out->bytes = p.DataBytes;
        out->data = p.Data;
        return r;
    }
    int enc_remove_before(unsigned num) { return sh->api->encoder_remove_before(enc, num); }

    // range calls (Stream::add_ranges): the originals of consecutive ids lie
    // at one stride in the device payload area
    std::vector<unsigned> lens;
    const unsigned* range_lens(unsigned firstId, unsigned count)
    {
        if (sh->cfg->payload_bytes)
            return nullptr;
        lens.resize(count);
        for (unsigned k = 0; k < count; ++k)
            lens[k] = scen::variable_bytes(firstId + k);
        return lens.data();
    }
    unsigned payload_bytes_of(unsigned id) const
    {
        return sh->cfg->payload_bytes ? sh->cfg->payload_bytes : scen::variable_bytes(id);
    }
    int enc_add_range(unsigned firstId, unsigned count, unsigned* firstNum, unsigned* added)
    {
        if (sh->frames || !sh->api->encoder_add_range) {   // (frames: datagrams one at a time)
            *added = 0;
            for (unsigned k = 0; k < count; ++k) {
                unsigned num = 0;
                const int r = enc_add(firstId + k, nullptr, payload_bytes_of(firstId + k), &num);
                if (r != 0)
                    return r;
                if (k == 0)
                    *firstNum = num;
                ++*added;
            }
            return 0;
        }
        const unsigned* l = range_lens(firstId, count);
        CallTimer ct(kEncAdd, count);
        return sh->api->encoder_add_range(enc, dev_payload(firstId), sh->stride, l, sh->cfg->payload_bytes, count,
                                          firstNum, added);
    }
    int dec_add_range(unsigned firstId, unsigned firstNum, unsigned count, int* results, unsigned* calls)
    {
        if (sh->frames || !sh->api->decoder_add_original_range) {
            *calls = 0;
            for (unsigned k = 0; k < count; ++k) {
                const int r = dec_add_original(firstId + k, (firstNum + k) & 0x3fffff, nullptr,
                                               payload_bytes_of(firstId + k));
                results[k] = r;
                ++*calls;
                if (r != 0 && r != 4)
                    return r;
            }
            return 0;
        }
        const unsigned* l = range_lens(firstId, count);
        static_assert(sizeof(SiameseResult) == sizeof(int), "result array");
        CallTimer ct(kDecAddOrig, count);
        return sh->api->decoder_add_original_range(dec, firstNum, dev_payload(firstId), sh->stride, l,
                                                   sh->cfg->payload_bytes, count,
                                                   reinterpret_cast<SiameseResult*>(results), calls);
    }
    std::vector<SiameseOriginalPacket> gets;
    int dec_get_range(unsigned firstNum, unsigned count, Pkt* out, unsigned* got)
    {
        if (sh->defer || !sh->api->decoder_get_range) {   // (deferred entries: one call each)
            *got = 0;
            for (unsigned k = 0; k < count; ++k) {
                const int r = dec_get((firstNum + k) & 0x3fffff, &out[k]);
                if (r != 0)
                    return r;
                ++*got;
            }
            return 0;
        }
        gets.resize(count);
        CallTimer ct(kDecGet, count);
        const int r = sh->api->decoder_get_range(dec, firstNum, count, gets.data(), got);
        for (unsigned k = 0; k < *got; ++k) {
            out[k].num = gets[k].PacketNum;
            out[k].bytes = gets[k].DataBytes;
            out[k].data = gets[k].Data;
            out[k].entry = nullptr;
        }
        return r;
    }

    uint64_t rec_token(const Rec& r)
    {
        // end-to-end mode: every recovery packet goes back to host memory
        if (sh->hashData || sh->e2e)
            push(Request{log, log->size(), r.pkt.DeviceData, r.bytes, flow, false, nullptr});
        return r.bytes;
    }
    uint64_t pkt_token(const Pkt& p, unsigned id, bool* ok)
    {
        if (sh->defer && p.entry && p.entry->DataBytes == 0) {
            // length and bytes arrive with the round's completion: the token
            // is written into the log then (resolve_requests).  (An entry the
            // call filled at once -- a packet not being solved -- is checked
            // right here like a plain one: no request to carry through the
            // main thread's collection.)
            push(Request{log, log->size(), nullptr, 0, id, true, ok, p.entry});
            return 0;
        }
        const unsigned bytes = p.entry ? p.entry->DataBytes : p.bytes;
        const void* data = p.entry ? p.entry->Data : p.data;
        const unsigned want = sh->cfg->payload_bytes ? sh->cfg->payload_bytes : scen::variable_bytes(id);
        if (bytes != want || !data) {
            if (std::getenv("SCENARIO_DEBUG"))
                std::fprintf(stderr, "pkt_token: id %u entry %d bytes %u want %u data %p\n", id,
                             p.entry != nullptr, bytes, want, data);
            *ok = false;
        } else if (sh->hashData || sh->verify || (sh->e2e && p.entry))
            // end-to-end mode copies back what exists only on the device: a
            // recovered original (a decode output); a delivered original that
            // arrived intact came from host memory, where the application
            // still has it
            push(Request{log, log->size(), data, bytes, id, true, ok});
        return bytes;
    }
    void push(Request r)
    {
        r.inFlight = &inFlight;
        ++inFlight;
        cur.push_back(r);
    }
    bool wants_yield_after_decode()
    {
        if (!sh->defer)
            return true;
        if (++decodes < sh->defer)
            return false;
        decodes = 0;
        return true;
    }
    bool wants_yield_after_encode() const { return sh->hashData; }
    bool outputs_final(const std::vector<Pkt>& v) const
    {
        for (const Pkt& p : v)
            if (!p.entry || !p.entry->Data)
                return false;
        return true;
    }
    /// Back to the freshly constructed state (a recycled job's codec slot).
    void reset()
    {
        enc = nullptr;
        dec = nullptr;
        cur.clear();
        inFlight = 0;
        decodes = 0;
        slabs.clear();
        slabUsed = kSlab;
        ahead.clear();
        aheadNext = 0;
        aheadFail = 0;
    }
};

using BatchStream = scen::Stream<BatchCodec, Rec, Pkt>;

// Wait for the oldest gather in flight, then check / hash its bytes.
void land_gather(Shared& sh)
{
    Shared::Gather g = std::move(sh.gathers.front());
    sh.gathers.pop_front();
    if (sh.api->gather_wait(g.ticket) != 0) {
        for (const Request& r : g.reqs)
            if (r.ok)
                *r.ok = false;
        ++sh.mismatches;
    } else {
        std::vector<uint8_t> expect;
        size_t off = 0;
        std::vector<SgpuFrame> frames;
        if (g.framed) {
            // the landed frame stream: one recovery frame per request, in order
            frames.resize(g.reqs.size());
            unsigned n = 0;
            if (sh.api->frames_parse(g.land.buf, g.bytes, frames.data(), (unsigned)frames.size(), &n) !=
                    Siamese_Success || n != g.reqs.size()) {
                for (const Request& r : g.reqs)
                    if (r.ok)
                        *r.ok = false;
                ++sh.mismatches;
                sh.landings.push_back(g.land);
                return;
            }
        }
        for (size_t i = 0; i < g.reqs.size(); ++i) {
            const Request& r = g.reqs[i];
            const uint8_t* d = g.land.buf + off;
            off += (r.bytes + 15) & ~(size_t)15;
            if (g.framed) {
                const SgpuFrame& f = frames[i];
                d = g.land.buf + f.Offset;
                if (f.Type != SGPU_FRAME_RECOVERY || f.Flow != r.id || f.Bytes != r.bytes)
                    ++sh.mismatches;
            }
            if (r.isPacket && (sh.verify || sh.hashData)) {
                expect.resize(r.bytes + 8);
                scen::fill_payload(r.id, expect.data(), r.bytes);
                ++sh.checked;
                if (std::memcmp(expect.data(), d, r.bytes) != 0) {
                    ++sh.mismatches;
                    *r.ok = false;
                    if (std::getenv("SCENARIO_DEBUG")) {
                        size_t at = 0;
                        while (at < r.bytes && expect[at] == d[at])
                            ++at;
                        std::fprintf(stderr, "mismatch: id %u bytes %u first differing byte %zu (deferred %d) dev %p\n",
                                     r.id, r.bytes, at, r.entry != nullptr, r.dev);
                    }
                }
            }
            if (sh.hashData)
                (*r.log)[r.pos] = scen::data_token(true, d, r.bytes);
        }
    }
    sh.landings.push_back(g.land);
}

void land_gathers(Shared& sh)
{
    while (!sh.gathers.empty())
        land_gather(sh);
}

// Resolve tokens whose data was produced by an already completed flush: one
// gather of all their device ranges into a pinned landing buffer (16-byte
// aligned ranges, one DMA), issued without waiting.  The requests come from
// completed submissions, so nothing waits for the flushes in flight, and the
// codecs owning the ranges may be driven on at once (later device work waits
// for the gather's reads).  Bytes that are checked or hashed are examined
// when the gather lands (land_gather).
void gather_requests(Shared& sh, std::vector<Request>& reqs, bool framed);

void resolve_requests(Shared& sh, std::vector<Request>& reqs)
{
    if (reqs.empty())
        return;
    // deferred outputs: their length and pointer are final now; a token
    // that needs no bytes is written here, the rest join the gather
    size_t keep = 0;
    for (size_t i = 0; i < reqs.size(); ++i) {
        Request r = reqs[i];
        --*r.inFlight;
        if (r.entry) {
            r.dev = r.entry->Data;
            r.bytes = r.entry->DataBytes;
            const unsigned want = sh.cfg->payload_bytes ? sh.cfg->payload_bytes : scen::variable_bytes(r.id);
            if (r.bytes != want || !r.dev) {
                if (std::getenv("SCENARIO_DEBUG"))
                    std::fprintf(stderr, "deferred token: id %u bytes %u want %u data %p\n", r.id, r.bytes,
                                 want, r.dev);
                *r.ok = false;
                if (!r.log->empty())
                    (*r.log)[r.pos] = r.bytes;
                continue;
            }
            if (!r.log->empty())
                (*r.log)[r.pos] = r.bytes;   // (the token without hash_data; land_gather hashes)
            if (!(sh.hashData || sh.verify || sh.e2e))
                continue;
        }
        reqs[keep++] = r;
    }
    reqs.resize(keep);
    if (reqs.empty())
        return;
    if (sh.frames) {
        // recovery packets leave as framed datagrams (sgpu_frames_send); the
        // recovered originals' bytes by a plain gather
        std::vector<Request> rec, pkt;
        for (const Request& r : reqs)
            (r.isPacket ? pkt : rec).push_back(r);
        reqs.clear();
        if (!rec.empty())
            gather_requests(sh, rec, true);
        if (!pkt.empty())
            gather_requests(sh, pkt, false);
        return;
    }
    gather_requests(sh, reqs, false);
}

void gather_requests(Shared& sh, std::vector<Request>& reqs, bool framed)
{
    std::vector<const void*> srcs;
    std::vector<unsigned> lens;
    size_t total = 0;
    for (const Request& r : reqs) {
        srcs.push_back(r.dev);
        lens.push_back(r.bytes);
        total += (r.bytes + 15) & ~(size_t)15;
        if (framed)
            total += 16;   // (a frame header, at most 8 bytes, can add one lane)
    }
    constexpr size_t kInFlight = 4;
    if (sh.gathers.size() >= kInFlight)
        land_gather(sh);
    // a free landing buffer that fits (the largest one otherwise, regrown)
    Shared::Landing land;
    size_t pick = sh.landings.size();
    for (size_t k = 0; k < sh.landings.size(); ++k)
        if (sh.landings[k].cap >= total + 16 && (pick == sh.landings.size() || sh.landings[k].cap < sh.landings[pick].cap))
            pick = k;
    if (pick < sh.landings.size()) {
        land = sh.landings[pick];
        sh.landings.erase(sh.landings.begin() + (long)pick);
    } else {
        if (!sh.landings.empty()) {
            sh.api->host_free(sh.landings.back().buf);
            sh.landings.pop_back();
        }
        land.cap = ((total + 16) + (8u << 20) - 1) & ~(size_t)((8u << 20) - 1);
        land.buf = (uint8_t*)sh.api->host_alloc(land.cap);
    }
    long long t = -1;
    size_t frameBytes = 0;
    if (land.buf && framed) {
        std::vector<SgpuRecoveryPacket> pk(reqs.size());
        std::vector<unsigned> flows(reqs.size());
        for (size_t i = 0; i < reqs.size(); ++i) {
            std::memset(&pk[i], 0, sizeof(pk[i]));
            pk[i].DeviceData = static_cast<const unsigned char*>(reqs[i].dev);
            pk[i].DataBytes = reqs[i].bytes;
            flows[i] = reqs[i].id;
        }
        t = sh.api->frames_send((unsigned)reqs.size(), pk.data(), flows.data(), land.buf, land.cap, &frameBytes);
    } else if (land.buf) {
        t = sh.api->gather_async((unsigned)reqs.size(), srcs.data(), lens.data(), land.buf);
    }
    if (t <= 0) {
        if (land.buf)
            sh.landings.push_back(land);
        for (const Request& r : reqs)
            if (r.ok)
                *r.ok = false;
        ++sh.mismatches;
        reqs.clear();
        return;
    }
    Shared::Gather g;
    g.ticket = t;
    g.land = land;
    g.framed = framed;
    g.bytes = frameBytes;
    if (sh.verify || sh.hashData || framed)
        g.reqs.swap(reqs);
    sh.gathers.push_back(std::move(g));
    reqs.clear();
    // SCENARIO_SYNC_GATHER=1: land every gather at once (debugging aid)
    static const bool syncGather = std::getenv("SCENARIO_SYNC_GATHER") != nullptr;
    if (syncGather)
        land_gathers(sh);
}

// fn(i) for i in [0, count), blocks of a few streams per pool task: on the
// library's host threads (sgpu_parallel_for) unless the run asked for its
// own thread count
template <class F>
void for_streams(Shared& sh, size_t count, const F& fn)
{
    // streams per pool task (SCENARIO_BLOCK, default 2): small tasks keep a
    // fork-join's tail short (same-box A/B, profiles/r2m_block_ab.txt:
    // 7.04-7.36 ms/step with 2, 7.17-7.85 with 1, 7.84-8.82 with 4)
    static const size_t kBlock = [] {
        const char* v = std::getenv("SCENARIO_BLOCK");
        const long b = v ? std::atol(v) : 2;
        return (size_t)(b > 0 ? b : 2);
    }();
    const size_t blocks = (count + kBlock - 1) / kBlock;
    auto body = [&](size_t b) {
        const uint64_t t0 = kCallTiming ? __builtin_ia32_rdtsc() : 0;
        const size_t end = std::min(count, (b + 1) * kBlock);
        for (size_t i = b * kBlock; i < end; ++i)
            fn(i);
        if (kCallTiming)
            call_counts().busy += __builtin_ia32_rdtsc() - t0;
    };
    struct Wall
    {
        uint64_t t0 = kCallTiming ? __builtin_ia32_rdtsc() : 0;
        ~Wall()
        {
            if (kCallTiming) {
                g_fjWall += __builtin_ia32_rdtsc() - t0;
                ++g_fjCount;
            }
        }
    } wall;
    if (sh.pool) {
        sh.pool->run(blocks, body);
        return;
    }
    using Body = decltype(body);
    sh.api->parallel_for((unsigned)blocks,
                         [](void* ctx, unsigned b) { (*static_cast<const Body*>(ctx))(b); },
                         (void*)&body);
}

// One job = one contiguous group of a step's streams.  Jobs flow through a
// pipeline so that the host work of one job overlaps the device work (and
// the library's launch and completion work) of the others: every iteration
// takes each active job in turn, resolves the tokens of its completed
// submissions, advances its streams to their next yield and submits again
// without waiting (sgpu_enqueue); a new job starts while the pipeline is
// shallow.  A job advances only once its last submission has completed
// (classic mode), or with up to two of its submissions in flight (deferred
// outputs, BatchOptions::defer: a single stream then keeps the GPU busy with
// one round while the host prepares the next).
struct Round
{
    long long ticket;
    std::vector<Request> reqs;   // tokens made in the round this submission closed
};

struct Job
{
    unsigned step = 0, begin = 0, end = 0;
    unsigned index = 0;             // step * groups + group
    bool fresh = false;             // codecs not created yet: the first advance does it
    bool second = false;            // e2e: the job's originals are in the second device copy
    std::vector<BatchCodec> codecs;
    std::unique_ptr<BatchStream[]> streams;
    // the job's own per-stream results: jobs of different steps run the
    // same streams and may be in flight together, so each keeps its own and
    // the last step's are copied out when it retires
    std::vector<StreamResult> res;
    std::vector<unsigned> live;     // indices into codecs/streams
    std::deque<Round> rounds;       // submitted, tokens not yet resolved (oldest first)
    std::vector<SgpuDecoder> decTable;   // frames: decoders by flow (the session's stream index)
};

int run_pipeline(Shared& sh, StreamResult* results, unsigned nsteps, uint64_t* rounds,
                 double* phase, uint64_t* payloadBytes)
{
    const Api& api = *sh.api;
    const ScenarioConfig* cfg = sh.cfg;
    const unsigned n = cfg->streams;
    const unsigned G = std::max(1u, std::min(sh.groups, n));
    // (SCENARIO_INFLIGHT overrides the deferred mode's depth: debugging aid)
    static const size_t kDeferDepth = [] {
        const char* v = std::getenv("SCENARIO_INFLIGHT");
        return (size_t)(v && std::atoi(v) > 0 ? std::atoi(v) : 2);
    }();
    const size_t inFlightPerJob = sh.defer ? kDeferDepth : 1;
    auto t = Clock::now();
    // SCENARIO_TIMELINE=1: one stderr line per phase (debugging aid)
    static const bool timeline = std::getenv("SCENARIO_TIMELINE") != nullptr;
    int curJob = -1;
    auto lap = [&](int k) {
        const auto now = Clock::now();
        phase[k] += std::chrono::duration<double>(now - t).count();
        if (timeline)
            std::fprintf(stderr, "tl %10.3f %8.3f ms  %s j%d\n",
                         std::chrono::duration<double>(t.time_since_epoch()).count() * 1e3,
                         std::chrono::duration<double>(now - t).count() * 1e3,
                         k == 0 ? "create" : k == 1 ? "step" : k == 2 ? "flush" : k == 3 ? "resolve" : "finish",
                         curJob);
        t = now;
    };
    auto take_cur = [](Job& J) {
        std::vector<Request> reqs;
        for (BatchCodec& c : J.codecs) {
            reqs.insert(reqs.end(), c.cur.begin(), c.cur.end());
            c.cur.clear();
        }
        return reqs;
    };
    // advance every live stream of J until it yields; finished streams free
    // their codecs right away (their state is still hot) unless tokens of
    // theirs still wait for device results; digests wait for the job's last
    // device bytes (retirement)
    // a stream's codecs and state, made on the thread that then steps it
    // (its first round: one fork-join instead of two, and the codec's memory
    // first touched by the core that works on it)
    auto start_stream = [&](Job& J, size_t i) {
        BatchCodec& c = J.codecs[i];
        c.reset();
        c.sh = &sh;
        c.payload = sh.frames ? (J.second ? sh.frameDev2 : sh.frameDev) : (J.second ? sh.payload2 : sh.payload);
        {
            CallTimer ct(kCreate);
            c.enc = api.encoder_create();
            c.dec = api.decoder_create();
        }
        c.flow = J.begin + (unsigned)i;
        if (sh.frames) {
            J.decTable[c.flow] = c.dec;   // (frames_recv reads only the entry of its frame's flow)
            c.decTable = J.decTable.data();
        }
        c.log = &J.streams[i].log;
        // the event log only feeds digests: timed bench steps run without it
        J.streams[i].logOn = sh.verify || sh.hashData || sh.digest;
        J.streams[i].init(cfg, &c, &J.res[i], cfg->first_stream + J.begin + (unsigned)i);
        if (!c.enc || !c.dec)
            J.streams[i].fail(2);
    };
    // Advance the live streams of several jobs in ONE fork-join (the first
    // listed first: a new job's long first rounds, then the short later
    // rounds of jobs whose submissions completed, which fill the fork-join's
    // tail instead of paying a fork-join of their own).
    std::vector<std::pair<Job*, unsigned>> items;
    auto advance_jobs = [&](Job* const* js, size_t count) {
        items.clear();
        for (size_t q = 0; q < count; ++q)
            for (unsigned i : js[q]->live)
                items.emplace_back(js[q], i);
        for_streams(sh, items.size(), [&](size_t k) {
            Job& J = *items[k].first;
            const unsigned i = items[k].second;
            if (J.fresh)
                start_stream(J, i);
            BatchStream& st = J.streams[i];
            while (!st.done())
                if (st.step())
                    break;
            BatchCodec& c = J.codecs[i];
            if (st.done() && c.inFlight == 0) {
                CallTimer ct(kFree);
                api.encoder_free(c.enc);
                api.decoder_free(c.dec);
                c.enc = nullptr;
                c.dec = nullptr;
            }
        });
        for (size_t q = 0; q < count; ++q) {
            Job& J = *js[q];
            J.fresh = false;
            J.live.erase(std::remove_if(J.live.begin(), J.live.end(),
                                        [&](unsigned i) { return J.streams[i].done(); }),
                         J.live.end());
        }
    };
    auto advance = [&](Job& J) {
        Job* one = &J;
        advance_jobs(&one, 1);
    };
    std::vector<std::unique_ptr<Job>> active;
    std::vector<std::unique_ptr<Job>> spareJobs;   // retired jobs, reused (their streams' vectors kept)
    // Resolve the tokens of J's completed rounds (oldest first).  -1 on a
    // device failure, else the number resolved.
    auto collect = [&](Job& J) {
        int got = 0;
        while (!J.rounds.empty()) {
            const int q = api.query(J.rounds.front().ticket);
            if (q < 0)
                return -1;
            if (q == 0)
                break;
            resolve_requests(sh, J.rounds.front().reqs);
            J.rounds.pop_front();
            ++got;
        }
        return got;
    };
    // Gather the tokens of every job's completed rounds.  Runs before each
    // submission: buffers a completed submission released (a decoder's
    // delivered slots, a freed codec's symbols) are free for any job's next
    // allocation, so the bytes a token names must be read before any later
    // submission, whose device work waits for the gather's reads, can
    // rewrite them.
    auto collect_all = [&]() {
        for (auto& a : active)
            if (collect(*a) < 0)
                return false;
        return true;
    };
    auto submit = [&](Job& J) {
        if (!collect_all())
            return false;
        Round r;
        r.reqs = take_cur(J);
        r.ticket = api.enqueue();
        if (timeline)
            std::fprintf(stderr, "tl submit j%d t%lld live %zu\n", curJob, r.ticket, J.live.size());
        ++*rounds;
        if (r.ticket < 0)
            return false;
        J.rounds.push_back(std::move(r));
        return true;
    };
    // one submission for the jobs advanced together: each job's round holds
    // its own tokens and the shared ticket
    auto submit_jobs = [&](Job* const* js, size_t count) {
        if (!collect_all())
            return false;
        for (size_t q = 0; q < count; ++q) {
            Round r;
            r.reqs = take_cur(*js[q]);
            js[q]->rounds.push_back(std::move(r));
        }
        const long long ticket = api.enqueue();
        if (timeline)
            std::fprintf(stderr, "tl submit j%d t%lld jobs %zu\n", curJob, ticket, count);
        ++*rounds;
        for (size_t q = 0; q < count; ++q) {
            if (ticket < 0)
                js[q]->rounds.pop_back();
            else
                js[q]->rounds.back().ticket = ticket;
        }
        return ticket >= 0;
    };
    auto dump = [&](Job& J) {
        // debugging aid: SCENARIO_DUMP="<stream index>:<path>" writes that
        // stream's event log (same format as scenario_run_capi's)
        const char* d = std::getenv("SCENARIO_DUMP");
        if (!d || J.step + 1 != nsteps)
            return;
        const unsigned idx = (unsigned)std::strtoul(d, nullptr, 10);
        const char* path = std::strchr(d, ':');
        if (path && idx >= J.begin && idx < J.end)
            if (FILE* f = std::fopen(path + 1, "w")) {
                for (uint64_t e : J.streams[idx - J.begin].log)
                    std::fprintf(f, "%016llx\n", (unsigned long long)e);
                std::fclose(f);
            }
    };

    const unsigned jobs = nsteps * G;
    const size_t depth = G + 1;   // jobs in flight
    unsigned next = 0;
    int rc = 0;
    // Host work is done whenever some is available: a job's completed rounds
    // are resolved, a job with room in flight is advanced (or retired), a new
    // job starts (round one, the bulk of a step's host work) while the
    // pipeline is shallow; the thread blocks only when none is possible.
    // Later rounds ride in the next new job's fork-join and submission
    // (classic mode, device-resident originals): a block-mode job's second
    // round (decode finish, frees) is ~1/3 of its first, and on its own paid a
    // whole fork-join's wake-ups and tail plus a submission
    // (SCENARIO_MERGE_ROUNDS=0: each round on its own, as before).
    // (=2: in the deferred-output mode too; a measuring aid)
    static const int kMergeRounds = [] {
        const char* v = std::getenv("SCENARIO_MERGE_ROUNDS");
        return v ? std::atoi(v) : 1;
    }();
    const bool merge = kMergeRounds > 0 && !sh.e2e && (inFlightPerJob == 1 || kMergeRounds == 2);
    std::vector<Job*> ready;   // (merge) jobs whose next round waits for the next fork-join
    auto run_ready = [&]() {
        if (ready.empty() || rc != 0)
            return;
        advance_jobs(ready.data(), ready.size());
        lap(1);
        if (!submit_jobs(ready.data(), ready.size()))
            rc = -3;
        lap(2);
        ready.clear();
    };
    while (rc == 0 && (next < jobs || !active.empty())) {
        bool did = false;
        ready.clear();
        for (size_t k = 0; k < active.size() && rc == 0;) {
            Job& J = *active[k];
            curJob = (int)(J.step * G + J.begin);
            const int got = collect(J);
            if (got < 0) {
                rc = -3;
                break;
            }
            if (got > 0) {
                did = true;
                lap(3);
            }
            if (!J.live.empty()) {
                if (J.rounds.size() < inFlightPerJob) {
                    did = true;
                    if (merge) {
                        ready.push_back(&J);
                    } else {
                        advance(J);
                        lap(1);
                        if (!submit(J))
                            rc = -3;
                        lap(2);
                    }
                }
                ++k;
                continue;
            }
            if (!J.rounds.empty()) {
                ++k;
                continue;
            }
            did = true;
            std::vector<Request> reqs = take_cur(J);   // (none: every round ends with a submission)
            resolve_requests(sh, reqs);
            if (sh.verify || sh.hashData)
                land_gathers(sh);   // (their requests point into the job's streams)
            auto finish_one = [&](size_t i) {
                J.streams[i].finish();
                CallTimer ct(kFree);
                api.encoder_free(J.codecs[i].enc);   // (null if freed already)
                api.decoder_free(J.codecs[i].dec);
                J.codecs[i].enc = nullptr;
                J.codecs[i].dec = nullptr;
            };
            // (without event logs there is no digest to hash, and codecs are
            // freed as their streams finish unless tokens of theirs were
            // still in flight then: no fork-join when nothing is left to do)
            bool work = sh.verify || sh.hashData || sh.digest;
            for (size_t i = 0; i < J.end - J.begin && !work; ++i)
                work = J.codecs[i].enc || J.codecs[i].dec;
            if (work)
                for_streams(sh, J.end - J.begin, finish_one);
            else
                for (size_t i = 0; i < J.end - J.begin; ++i)
                    finish_one(i);
            for (const StreamResult& r : J.res)
                *payloadBytes += r.payload_bytes;
            if (J.step + 1 == nsteps)
                std::copy(J.res.begin(), J.res.end(), results + J.begin);
            dump(J);
            spareJobs.push_back(std::move(active[k]));   // (its vectors are reused by a later job)
            active.erase(active.begin() + (long)k);
            lap(4);
        }
        // e2e: a job's device copy of its originals is overwritten by the job
        // two steps later (the copies alternate by step); that job starts
        // only once the earlier one has retired
        auto copy_busy = [&](unsigned idx) {
            if (!sh.e2e || idx < 2 * G)
                return false;
            for (const auto& a : active)
                if (a->index == idx - 2 * G)
                    return true;
            return false;
        };
        if (rc == 0 && next < jobs && active.size() < depth && !copy_busy(next)) {
            did = true;
            std::unique_ptr<Job> jp;
            if (!spareJobs.empty()) {
                jp = std::move(spareJobs.back());
                spareJobs.pop_back();
            } else {
                jp.reset(new Job);
            }
            Job& J = *jp;
            J.rounds.clear();
            J.live.clear();
            J.step = next / G;
            const unsigned g = next % G;
            J.begin = (unsigned)((uint64_t)n * g / G);
            J.end = (unsigned)((uint64_t)n * (g + 1) / G);
            J.index = next;
            curJob = (int)next;
            ++next;
            // e2e: the originals arrive in pinned host memory with each job,
            // into one of two device copies that alternate by step: only the
            // job's own streams' originals, so its device work waits for its
            // slice alone while the next slices are still on the bus.  The
            // copy runs on the library's staging stream beside the device
            // work in flight; the submissions after it wait for it.
            const bool second = sh.e2e && (J.step & 1u);
            if (sh.e2e) {
                // (frames: the job's slice of the framed ring instead)
                const size_t stride = sh.frames ? sh.fstride : sh.stride;
                uint8_t* dev = sh.frames ? (second ? sh.frameDev2 : sh.frameDev) : (second ? sh.devBase2 : sh.devBase);
                const uint8_t* host = sh.frames ? sh.frameHost : sh.hostPayload;
                const size_t per = (size_t)cfg->originals * stride;
                const size_t off = (size_t)J.begin * per, len = (size_t)(J.end - J.begin) * per;
                if (api.h2d_async(dev + off, host + off, len) != 0) {
                    rc = -3;
                    break;
                }
            }
            const unsigned cnt = J.end - J.begin;
            if (J.codecs.size() != cnt || !J.streams) {
                J.codecs.clear();
                J.codecs.resize(cnt);
                J.streams.reset(new BatchStream[cnt]);
            }
            J.res.assign(cnt, StreamResult{});
            if (sh.frames)
                J.decTable.assign(n, nullptr);
            J.second = second;
            J.fresh = true;   // (the codecs are made by the first advance, start_stream)
            for (unsigned i = 0; i < cnt; ++i)
                J.live.push_back(i);
            lap(0);
            if (merge) {
                ready.insert(ready.begin(), &J);   // (its first round leads the fork-join)
                run_ready();
            } else {
                advance(J);
                lap(1);
                if (!submit(J))
                    rc = -3;
                lap(2);
            }
            active.push_back(std::move(jp));
        }
        run_ready();   // (later rounds with no new job to ride with)
        if (rc == 0 && !did && !active.empty()) {
            // nothing to do until the oldest round in flight completes
            for (auto& a : active)
                if (!a->rounds.empty()) {
                    if (api.wait(a->rounds.front().ticket) != 0)
                        rc = -3;
                    break;
                }
            lap(2);
        }
    }
    if (api.flush() != 0)
        rc = -3;
    lap(2);
    land_gathers(sh);   // every output is in host memory before the run ends
    lap(3);
    return rc;
}

} // namespace

namespace {

struct Session
{
    Api* api;
    ScenarioConfig cfg;
    uint8_t* dev = nullptr;
    size_t payloadBytes = 0;
    Shared sh;
    double setupSeconds = 0;
};

Api g_api;
bool g_loaded = false;

} // namespace

extern "C" __attribute__((visibility("default")))
void* scenario_batch_open(const char* lib, const ScenarioConfig* cfg, int device)
{
    if (!g_loaded) {
        if (!load_api(lib, g_api))
            return nullptr;
        g_loaded = true;
    }
    if (g_api.init(device) != 0)
        return nullptr;
    // Application-side allocator tuning: every step creates and frees
    // thousands of codecs; keep freed heap memory in the process instead of
    // returning it to the kernel and faulting it back in on the next step.
    mallopt(M_MMAP_THRESHOLD, 32 << 20);
    mallopt(M_TRIM_THRESHOLD, 1 << 30);
    mallopt(M_TOP_PAD, 64 << 20);
    Session* ss = new Session;
    ss->api = &g_api;
    ss->cfg = *cfg;
    const ScenarioConfig* c = &ss->cfg;

    // Stage every original of every stream in HBM (untimed).
    const auto t0 = Clock::now();
    const size_t total = (size_t)c->streams * c->originals;
    const unsigned maxBytes = c->payload_bytes ? c->payload_bytes : 1200;
    const size_t stride = (maxBytes + 63) & ~(size_t)63;
    ss->dev = (uint8_t*)g_api.device_alloc(total * stride);
    if (!ss->dev) {
        delete ss;
        return nullptr;
    }
    ss->payloadBytes = total * stride;
    const size_t chunkPackets = std::max<size_t>(1, (size_t)(64u << 20) / stride);
    std::vector<uint8_t> host(chunkPackets * stride);
    for (size_t base = 0; base < total; base += chunkPackets) {
        const size_t cnt = std::min(chunkPackets, total - base);
        for (size_t k = 0; k < cnt; ++k) {
            const unsigned id = (unsigned)((size_t)c->first_stream * c->originals + base + k);
            const unsigned b = c->payload_bytes ? c->payload_bytes : scen::variable_bytes(id);
            scen::fill_payload(id, host.data() + k * stride, b);
        }
        g_api.h2d(ss->dev + base * stride, host.data(), cnt * stride);
    }
    // payload ids are global; offset the base so an id indexes it directly
    ss->sh.api = &g_api;
    ss->sh.cfg = c;
    ss->sh.payload = ss->dev - (size_t)c->first_stream * c->originals * stride;
    ss->sh.stride = stride;
    ss->sh.hashData = c->hash_data != 0;
    ss->setupSeconds = std::chrono::duration<double>(Clock::now() - t0).count();
    return ss;
}

extern "C" __attribute__((visibility("default")))
int scenario_batch_run(void* session, StreamResult* results, const BatchOptions* opt,
                       BatchReport* report)
{
    Session* ss = (Session*)session;
    const Api& api = *ss->api;
    Shared& sh = ss->sh;
    std::memset(report, 0, sizeof(*report));
    report->setup_seconds = ss->setupSeconds;
    sh.checked = sh.mismatches = 0;
    sh.e2e = opt->e2e != 0;
    if (sh.e2e && !sh.hostPayload) {
        // a pinned host image of the device payload area, and a second
        // device copy for alternate steps (untimed)
        sh.payloadBytes = ss->payloadBytes;
        sh.devBase = ss->dev;
        sh.devBase2 = (uint8_t*)api.device_alloc(sh.payloadBytes);
        sh.hostPayload = (uint8_t*)api.host_alloc(sh.payloadBytes);
        if (!sh.hostPayload || !sh.devBase2)
            return -2;
        sh.payload2 = sh.devBase2 + (sh.payload - ss->dev);
        const ScenarioConfig* c = &ss->cfg;
        for (size_t k = 0; k < (size_t)c->streams * c->originals; ++k) {
            const unsigned id = (unsigned)((size_t)c->first_stream * c->originals + k);
            const unsigned b = c->payload_bytes ? c->payload_bytes : scen::variable_bytes(id);
            scen::fill_payload(id, sh.hostPayload + k * sh.stride, b);
        }
    }
    sh.frames = sh.e2e && opt->frames != 0;
    if (sh.frames && !sh.frameHost) {
        // every original of the session as a framed datagram (siamese_gpu.h)
        // at a fixed stride in a pinned ring, and two device copies (untimed)
        const ScenarioConfig* c = &ss->cfg;
        const unsigned maxBytes = c->payload_bytes ? c->payload_bytes : 1200;
        sh.fstride = (api.frame_header_bytes(SGPU_FRAME_ORIGINAL, maxBytes) + maxBytes + 15) & ~(size_t)15;
        const size_t total = (size_t)c->streams * c->originals;
        sh.frameBytes = total * sh.fstride;
        sh.idBase = (uint64_t)c->first_stream * c->originals;
        sh.frameHost = (uint8_t*)api.host_alloc(sh.frameBytes);
        sh.frameDev = (uint8_t*)api.device_alloc(sh.frameBytes);
        sh.frameDev2 = (uint8_t*)api.device_alloc(sh.frameBytes);
        if (!sh.frameHost || !sh.frameDev || !sh.frameDev2)
            return -2;
        std::memset(sh.frameHost, 0, sh.frameBytes);
        for (size_t k = 0; k < total; ++k) {
            const unsigned id = (unsigned)(sh.idBase + k);
            const unsigned b = c->payload_bytes ? c->payload_bytes : scen::variable_bytes(id);
            uint8_t* f = sh.frameHost + k * sh.fstride;
            // (PacketNum: the stream's k-th original; rewritten when it is sent)
            const unsigned h = api.frame_write_header(SGPU_FRAME_ORIGINAL, (unsigned)(k / c->originals),
                                                      (unsigned)(k % c->originals), b, f);
            scen::fill_payload(id, f + h, b);
        }
    }
    int rc = 0;
    // warm-up runs one at a time (the first may verify every byte); then all
    // timed steps as one pipeline, so one step's device tail overlaps the
    // next step's host work
    const unsigned passes = opt->warmup + (opt->steps ? 1 : 0);
    for (unsigned r = 0; r < passes && rc == 0; ++r) {
        const bool timed = r >= opt->warmup;
        sh.verify = opt->verify && r == 0;
        sh.digest = opt->digest != 0;
        // streams run on the library's host threads unless a count is requested
        if (opt->threads == 0)
            sh.pool.reset();
        else if (!sh.pool || sh.pool->size() != opt->threads)
            sh.pool.reset(new sgpu::WorkerPool(opt->threads));
        sh.groups = opt->groups ? opt->groups : 1;
        sh.defer = opt->defer;
        sh.deviceGe = opt->device_ge && !opt->defer && api.decode_device;
        uint64_t rounds = 0, payload = 0;
        double phase[5] = {0, 0, 0, 0, 0};
        // headroom over the warm-up's high-water mark, so the working set's
        // run-to-run variation in a pipelined loop takes reserved chunks
        // instead of hipMalloc calls inside the timed steps (untimed)
        if (timed && api.arena_reserve(api.arena_bytes() / 4) != 0)
            return -2;
        uint64_t e0[kEngineStats + 1], e1[kEngineStats + 1];
        auto stats = [&](uint64_t* e) {
            for (int k = 15; k < kEngineStats; ++k)
                e[k] = 0;
            if (api.engine_stats_ex)
                api.engine_stats_ex(e, kEngineStats);
            else
                api.engine_stats(e);   // (an older build: no k_ldpc bytes)
            e[kEngineStats] = api.arena_bytes();
        };
        stats(e0);
        api.timing(timed && !opt->no_timing ? 1 : 0, 1, nullptr, nullptr);
        if (api.measure_unique)
            api.measure_unique(opt->unique ? 1 : 0);
        const auto t1 = Clock::now();
        rc = run_pipeline(sh, results, timed ? opt->steps : 1, &rounds, phase, &payload);
        const double dt = std::chrono::duration<double>(Clock::now() - t1).count();
        if (api.measure_unique)
            api.measure_unique(0);
        double execMs = 0, totalMs = 0, kernelMs[5] = {0, 0, 0, 0, 0};
        if (api.timing_kernels)
            api.timing_kernels(kernelMs, 5);
        api.timing(0, 1, &execMs, &totalMs);
        stats(e1);
        if (timed) {
            report->seconds += dt;
            report->device_ms += totalMs;
            report->exec_ms += execMs;
            for (int k = 0; k < 5; ++k)
                report->kernel_ms[k] += kernelMs[k];
            report->rounds += rounds;
            report->payload_bytes += payload;
            for (int k = 0; k < 5; ++k)
                report->phase_seconds[k] += phase[k];
            for (int k = 0; k <= kEngineStats; ++k)
                report->engine[k] += e1[k] - e0[k];
        }
    }
    report->checked = sh.checked;
    report->mismatches = sh.mismatches;
    print_calls();
    return rc;
}

extern "C" __attribute__((visibility("default")))
void scenario_batch_close(void* session)
{
    Session* ss = (Session*)session;
    if (!ss)
        return;
    ss->api->device_free(ss->dev);
    if (ss->sh.devBase2)
        ss->api->device_free(ss->sh.devBase2);
    if (ss->sh.hostPayload)
        ss->api->host_free(ss->sh.hostPayload);
    if (ss->sh.frameHost)
        ss->api->host_free(ss->sh.frameHost);
    if (ss->sh.frameDev)
        ss->api->device_free(ss->sh.frameDev);
    if (ss->sh.frameDev2)
        ss->api->device_free(ss->sh.frameDev2);
    land_gathers(ss->sh);
    for (const Shared::Landing& l : ss->sh.landings)
        ss->api->host_free(l.buf);
    delete ss;
}

extern "C" __attribute__((visibility("default")))
int scenario_run_batch(const char* lib, const ScenarioConfig* cfg, StreamResult* results,
                       const BatchOptions* opt, BatchReport* report)
{
    void* s = scenario_batch_open(lib, cfg, opt->device);
    if (!s)
        return -2;
    const int rc = scenario_batch_run(s, results, opt, report);
    scenario_batch_close(s);
    return rc;
}
