// harness/scenario_capi.cpp -- sequential per-call driver for ANY siamese.h
// implementation, loaded with dlopen(RTLD_LOCAL) so the upstream reference
// (oracle/_ref/libsiamese_ref.so) and the MI355X library
// (siamese_amd/libsiamese_amd.so) can be driven side by side in one process.
//
// Exported (ctypes):
//   int scenario_run_capi(const char* lib, const ScenarioConfig* cfg,
//                         StreamResult* results, unsigned threads,
//                         double* seconds_out, const char* event_log_path)
// Only the codec calls are timed (payload generation and the loss channel are
// excluded), matching BASELINE.md section 3.
#include "scenario.h"
#include "../include/siamese.h"

#include <dlfcn.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

namespace {

struct CApi
{
    int (*init_)(int);
    SiameseEncoder (*encoder_create)();
    void (*encoder_free)(SiameseEncoder);
    SiameseResult (*encoder_add)(SiameseEncoder, SiameseOriginalPacket*);
    SiameseResult (*encoder_remove_before)(SiameseEncoder, unsigned);
    SiameseResult (*encode)(SiameseEncoder, SiameseRecoveryPacket*);
    SiameseDecoder (*decoder_create)();
    void (*decoder_free)(SiameseDecoder);
    SiameseResult (*decoder_add_original)(SiameseDecoder, const SiameseOriginalPacket*);
    SiameseResult (*decoder_add_recovery)(SiameseDecoder, const SiameseRecoveryPacket*);
    SiameseResult (*decoder_get)(SiameseDecoder, SiameseOriginalPacket*);
    SiameseResult (*decoder_is_ready)(SiameseDecoder);
    SiameseResult (*decode)(SiameseDecoder, SiameseOriginalPacket**, unsigned*);
};

template <class F>
bool bind(void* h, F& fn, const char* name)
{
    fn = reinterpret_cast<F>(dlsym(h, name));
    return fn != nullptr;
}

bool load_api(const char* path, CApi& api)
{
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        std::fprintf(stderr, "scenario: dlopen(%s) failed: %s\n", path, dlerror());
        return false;
    }
    return bind(h, api.init_, "siamese_init_") &&
           bind(h, api.encoder_create, "siamese_encoder_create") &&
           bind(h, api.encoder_free, "siamese_encoder_free") &&
           bind(h, api.encoder_add, "siamese_encoder_add") &&
           bind(h, api.encoder_remove_before, "siamese_encoder_remove_before") &&
           bind(h, api.encode, "siamese_encode") &&
           bind(h, api.decoder_create, "siamese_decoder_create") &&
           bind(h, api.decoder_free, "siamese_decoder_free") &&
           bind(h, api.decoder_add_original, "siamese_decoder_add_original") &&
           bind(h, api.decoder_add_recovery, "siamese_decoder_add_recovery") &&
           bind(h, api.decoder_get, "siamese_decoder_get") &&
           bind(h, api.decoder_is_ready, "siamese_decoder_is_ready") &&
           bind(h, api.decode, "siamese_decode");
}

struct Rec
{
    unsigned bytes = 0;
    const unsigned char* data = nullptr;
};

struct Pkt
{
    unsigned num = 0, bytes = 0;
    const unsigned char* data = nullptr;
};

using Clock = std::chrono::steady_clock;

// per call kind: count and seconds (SCENARIO_CAPI_CALLS=1 prints them per
// stream range on stderr; profiling aid)
enum CallKind { kCreate, kEncAdd, kEncode, kDecAddOrig, kDecAddRec, kIsReady, kDecode, kDecGet, kRemove, kFree, kKinds };
const char* const kCallNames[kKinds] = {"create", "enc_add", "encode", "dec_add_orig", "dec_add_rec",
                                        "is_ready", "decode", "dec_get", "remove_before", "free"};

struct Timer
{
    double& acc;
    double* kind;
    Clock::time_point t0;
    explicit Timer(double& a, double* k = nullptr) : acc(a), kind(k), t0(Clock::now()) {}
    ~Timer()
    {
        const double d = std::chrono::duration<double>(Clock::now() - t0).count();
        acc += d;
        if (kind) {
            kind[0] += 1;
            kind[1] += d;
        }
    }
};

struct CapiCodec
{
    const CApi* api = nullptr;
    const ScenarioConfig* cfg = nullptr;
    SiameseEncoder enc = nullptr;
    SiameseDecoder dec = nullptr;
    std::vector<uint8_t> expect;
    double seconds = 0;
    double calls[kKinds][2] = {};

    bool needs_host_payload() const { return true; }

    int enc_add(unsigned, const uint8_t* data, unsigned bytes, unsigned* num)
    {
        SiameseOriginalPacket p;
        p.PacketNum = 0;
        p.Data = data;
        p.DataBytes = bytes;
        int r;
        {
            Timer t(seconds, calls[kEncAdd]);
            r = api->encoder_add(enc, &p);
        }
        *num = p.PacketNum;
        return r;
    }
    int encode(Rec* rec)
    {
        SiameseRecoveryPacket r{};
        int res;
        {
            Timer t(seconds, calls[kEncode]);
            res = api->encode(enc, &r);
        }
        rec->bytes = r.DataBytes;
        rec->data = r.Data;
        return res;
    }
    int dec_add_original(unsigned, unsigned num, const uint8_t* data, unsigned bytes)
    {
        SiameseOriginalPacket p;
        p.PacketNum = num;
        p.Data = data;
        p.DataBytes = bytes;
        Timer t(seconds, calls[kDecAddOrig]);
        return api->decoder_add_original(dec, &p);
    }
    int dec_add_recovery(const Rec& rec)
    {
        SiameseRecoveryPacket r;
        r.Data = rec.data;
        r.DataBytes = rec.bytes;
        Timer t(seconds, calls[kDecAddRec]);
        return api->decoder_add_recovery(dec, &r);
    }
    int is_ready()
    {
        Timer t(seconds, calls[kIsReady]);
        return api->decoder_is_ready(dec);
    }
    int decode(std::vector<Pkt>* out)
    {
        SiameseOriginalPacket* pkts = nullptr;
        unsigned count = 0;
        int r;
        {
            Timer t(seconds, calls[kDecode]);
            r = api->decode(dec, &pkts, &count);
        }
        if (r == 0)
            for (unsigned i = 0; i < count; ++i)
                out->push_back(Pkt{pkts[i].PacketNum, pkts[i].DataBytes, pkts[i].Data});
        return r;
    }
    int dec_get(unsigned num, Pkt* out)
    {
        SiameseOriginalPacket p;
        p.PacketNum = num;
        p.Data = nullptr;
        p.DataBytes = 0;
        int r;
        {
            Timer t(seconds, calls[kDecGet]);
            r = api->decoder_get(dec, &p);
        }
        out->num = num;
        out->bytes = p.DataBytes;
        out->data = p.Data;
        return r;
    }
    int enc_remove_before(unsigned num)
    {
        Timer t(seconds, calls[kRemove]);
        return api->encoder_remove_before(enc, num);
    }
    // range calls as loops of the single calls (Stream::add_ranges)
    std::vector<uint8_t> pbuf;
    const uint8_t* payload(unsigned id, unsigned* bytes)
    {
        *bytes = cfg->payload_bytes ? cfg->payload_bytes : scen::variable_bytes(id);
        pbuf.resize(*bytes + 8);
        scen::fill_payload(id, pbuf.data(), *bytes);
        return pbuf.data();
    }
    int enc_add_range(unsigned firstId, unsigned count, unsigned* firstNum, unsigned* added)
    {
        *added = 0;
        *firstNum = 0;
        for (unsigned k = 0; k < count; ++k) {
            unsigned bytes = 0, num = 0;
            const uint8_t* d = payload(firstId + k, &bytes);
            const int r = enc_add(firstId + k, d, bytes, &num);
            if (r != 0)
                return r;
            if (k == 0)
                *firstNum = num;
            ++*added;
        }
        return 0;
    }
    int dec_add_range(unsigned firstId, unsigned firstNum, unsigned count, int* results, unsigned* calls)
    {
        *calls = 0;
        for (unsigned k = 0; k < count; ++k) {
            unsigned bytes = 0;
            const uint8_t* d = payload(firstId + k, &bytes);
            const int r = dec_add_original(firstId + k, (firstNum + k) & 0x3fffff, d, bytes);
            results[k] = r;
            ++*calls;
            if (r != 0 && r != 4)
                return r;
        }
        return 0;
    }
    int dec_get_range(unsigned firstNum, unsigned count, Pkt* out, unsigned* got)
    {
        *got = 0;
        for (unsigned k = 0; k < count; ++k) {
            const int r = dec_get((firstNum + k) & 0x3fffff, &out[k]);
            if (r != 0)
                return r;
            ++*got;
        }
        return 0;
    }

    uint64_t rec_token(const Rec& rec) { return scen::data_token(cfg->hash_data, rec.data, rec.bytes); }
    uint64_t pkt_token(const Pkt& p, unsigned id, bool* ok)
    {
        expect.resize(p.bytes + 8);
        scen::fill_payload(id, expect.data(), p.bytes);
        const unsigned want = cfg->payload_bytes ? cfg->payload_bytes : scen::variable_bytes(id);
        if (!p.data || p.bytes != want || std::memcmp(expect.data(), p.data, p.bytes) != 0)
            *ok = false;
        return p.data ? scen::data_token(cfg->hash_data, p.data, p.bytes) : 0;
    }
    void encode_hint(unsigned) {}   // (siamese.h encodes one packet per call)
    bool wants_yield_after_decode() const { return false; }
    bool outputs_final(const std::vector<Pkt>&) const { return true; }
    bool wants_yield_after_encode() const { return false; }
};

using CapiStream = scen::Stream<CapiCodec, Rec, Pkt>;

void run_range(const CApi* api, const ScenarioConfig* cfg, StreamResult* results, unsigned begin,
               unsigned end, double* seconds, FILE* log)
{
    for (unsigned s = begin; s < end; ++s) {
        CapiCodec codec;
        codec.api = api;
        codec.cfg = cfg;
        {
            Timer t(codec.seconds, codec.calls[kCreate]);
            codec.enc = api->encoder_create();
            codec.dec = api->decoder_create();
        }
        CapiStream st;
        st.init(cfg, &codec, &results[s], cfg->first_stream + s);
        if (!codec.enc || !codec.dec)
            st.fail(2);
        while (!st.done())
            st.step();
        st.finish();
        {
            Timer t(codec.seconds, codec.calls[kFree]);
            api->encoder_free(codec.enc);
            api->decoder_free(codec.dec);
        }
        if (log && s == begin) {
            for (uint64_t e : st.log)
                std::fprintf(log, "%016llx\n", (unsigned long long)e);
        }
        *seconds += codec.seconds;
        static const bool printCalls = std::getenv("SCENARIO_CAPI_CALLS") != nullptr;
        if (printCalls)
            for (unsigned k = 0; k < kKinds; ++k)
                if (codec.calls[k][0] > 0)
                    std::fprintf(stderr, "capi %-14s %6.0f calls %9.1f us  %7.2f us/call\n", kCallNames[k],
                                 codec.calls[k][0], codec.calls[k][1] * 1e6, codec.calls[k][1] * 1e6 / codec.calls[k][0]);
    }
}

} // namespace

extern "C" __attribute__((visibility("default")))
int scenario_run_capi(const char* lib, const ScenarioConfig* cfg, StreamResult* results,
                      unsigned threads, double* seconds_out, const char* event_log_path)
{
    CApi api;
    if (!load_api(lib, api))
        return -1;
    if (api.init_(SIAMESE_VERSION) != 0)
        return -2;
    if (threads == 0)
        threads = 1;
    if (threads > cfg->streams)
        threads = cfg->streams ? cfg->streams : 1;

    FILE* log = nullptr;
    if (event_log_path && event_log_path[0])
        log = std::fopen(event_log_path, "w");

    std::vector<double> secs(threads, 0.0);
    const auto t0 = Clock::now();
    if (threads == 1) {
        run_range(&api, cfg, results, 0, cfg->streams, &secs[0], log);
    } else {
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < threads; ++t) {
            const unsigned b = (unsigned)((uint64_t)cfg->streams * t / threads);
            const unsigned e = (unsigned)((uint64_t)cfg->streams * (t + 1) / threads);
            pool.emplace_back(run_range, &api, cfg, results, b, e, &secs[t], t == 0 ? log : nullptr);
        }
        for (auto& th : pool)
            th.join();
    }
    const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
    if (log)
        std::fclose(log);
    // Codec-call time: one thread's sum, or with several threads (each
    // driving its own streams at once) the longest any of them spent in codec
    // calls.  Payload generation and checking (harness work) are outside it.
    (void)wall;
    double longest = 0;
    for (double s : secs)
        longest = std::max(longest, s);
    if (seconds_out)
        *seconds_out = longest;
    return 0;
}
