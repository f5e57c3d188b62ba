// batch.cpp -- siamese_gpu.h: the device-resident batch API.  Same control
// plane as the drop-in API; instances keep no host mirrors and never wait
// for the device until sgpu_flush().
#define SIAMESE_BUILDING
#include "../../include/siamese_gpu.h"

#include "backend.h"
#include "decoder.h"
#include "frames.h"
#include "encoder.h"
#include "engine.h"
#include "objpool.h"
#include "pool.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

using namespace sgpu;

namespace {

bool g_batchReady = false;

struct BatchEncoder
{
    EncoderCore core{Engine::global(), false};
};

struct BatchDecoder
{
    DecoderCore core{Engine::global(), false};
};

inline BatchEncoder* BE(SgpuEncoder e) { return reinterpret_cast<BatchEncoder*>(e); }
inline BatchDecoder* BD(SgpuDecoder d) { return reinterpret_cast<BatchDecoder*>(d); }
using Lock = std::lock_guard<std::mutex>;

} // namespace

extern "C" {

SIAMESE_EXPORT int sgpu_init(int device)
{
    if (!gf_init())
        return Siamese_Disabled;
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    const char* err = "unknown";
    if (!eng->init(device, &err)) {
        std::fprintf(stderr, "siamese_amd: initialisation failed: %s\n", err);
        return Siamese_Disabled;
    }
    g_batchReady = true;
    return Siamese_Success;
}

SIAMESE_EXPORT SgpuEncoder sgpu_encoder_create(void)
{
    if (!g_batchReady)
        return nullptr;
    // (storage recycled per thread: objpool.h RawPool)
    void* m = RawPool<BatchEncoder>::get();
    return m ? reinterpret_cast<SgpuEncoder>(new (m) BatchEncoder) : nullptr;
}

SIAMESE_EXPORT void sgpu_encoder_free(SgpuEncoder encoder)
{
    if (!encoder)
        return;
    BE(encoder)->~BatchEncoder();
    RawPool<BatchEncoder>::put(BE(encoder));
}

SIAMESE_EXPORT SiameseResult sgpu_encoder_add(SgpuEncoder encoder, const void* deviceData, unsigned bytes,
                                              unsigned* packetNumOut)
{
    if (!encoder || !deviceData || bytes == 0 || bytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    SiameseOriginalPacket p;
    p.PacketNum = 0;
    p.Data = (const unsigned char*)deviceData;
    p.DataBytes = bytes;
    const SiameseResult r = BE(encoder)->core.add(p, (uint64_t)(uintptr_t)deviceData);
    if (packetNumOut)
        *packetNumOut = p.PacketNum;
    return r;
}

SIAMESE_EXPORT SiameseResult sgpu_encoder_add_range(SgpuEncoder encoder, const void* deviceData, size_t stride,
                                                    const unsigned* bytes, unsigned fixedBytes, unsigned count,
                                                    unsigned* firstPacketNumOut, unsigned* addedOut)
{
    if (addedOut)
        *addedOut = 0;
    if (!encoder || (!deviceData && count) || stride > 0xffffffffu || (count > 1 && stride == 0))
        return Siamese_InvalidInput;
    unsigned first = 0, added = 0;
    const SiameseResult r = BE(encoder)->core.add_range((uint64_t)(uintptr_t)deviceData, (uint32_t)stride, bytes,
                                                        fixedBytes, count, &first, &added);
    if (firstPacketNumOut)
        *firstPacketNumOut = first;
    if (addedOut)
        *addedOut = added;
    return r;
}

SIAMESE_EXPORT SiameseResult sgpu_encoder_remove_before(SgpuEncoder encoder, unsigned firstKept)
{
    if (!encoder || firstKept > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    BE(encoder)->core.remove_before(firstKept);
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult sgpu_encode(SgpuEncoder encoder, SgpuRecoveryPacket* out)
{
    if (!encoder || !out)
        return Siamese_InvalidInput;
    EncoderCore& core = BE(encoder)->core;
    EncodeOut o;
    const SiameseResult r = core.encode(o);
    if (r != Siamese_Success) {
        out->DataBytes = 0;
        return r;
    }
    out->DeviceData = o.buf.ptr;
    out->DataBytes = o.bytes;
    out->FooterBytes = o.footerBytes;
    std::memcpy(out->Footer, o.footer, sizeof(out->Footer));
    std::memcpy(out->Head, o.head, sizeof(out->Head));
    out->Producer = &core.program();
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult sgpu_encode_range(SgpuEncoder encoder, SgpuRecoveryPacket* out, unsigned count,
                                               unsigned* producedOut)
{
    if (producedOut)
        *producedOut = 0;
    if (!encoder || (!out && count) || !producedOut)
        return Siamese_InvalidInput;
    EncoderCore& core = BE(encoder)->core;
    // (EncodeOut is larger than the caller's records: encode in chunks)
    constexpr unsigned kChunk = 64;
    EncodeOut o[kChunk];
    SiameseResult r = Siamese_Success;
    unsigned done = 0;
    while (done < count && r == Siamese_Success) {
        const unsigned n = std::min(kChunk, count - done);
        unsigned made = 0;
        // (chunks after the first must keep the packets of the earlier ones:
        // one encode_range call per sgpu_encode_range, so chunking is by
        // hand below when count > kChunk)
        if (done == 0)
            r = core.encode_range(o, n, &made);
        else
            r = core.encode_range_more(o, n, &made);
        for (unsigned k = 0; k < made; ++k) {
            SgpuRecoveryPacket& p = out[done + k];
            p.DeviceData = o[k].buf.ptr;
            p.DataBytes = o[k].bytes;
            p.FooterBytes = o[k].footerBytes;
            std::memcpy(p.Footer, o[k].footer, sizeof(p.Footer));
            std::memcpy(p.Head, o[k].head, sizeof(p.Head));
            p.Producer = &core.program();
        }
        done += made;
        if (made < n && r == Siamese_Success)
            break;
    }
    if (r != Siamese_Success && done < count)
        out[done].DataBytes = 0;
    *producedOut = done;
    return r;
}

SIAMESE_EXPORT SgpuDecoder sgpu_decoder_create(void)
{
    if (!g_batchReady)
        return nullptr;
    void* m = RawPool<BatchDecoder>::get();
    return m ? reinterpret_cast<SgpuDecoder>(new (m) BatchDecoder) : nullptr;
}

SIAMESE_EXPORT void sgpu_decoder_free(SgpuDecoder decoder)
{
    if (!decoder)
        return;
    BD(decoder)->~BatchDecoder();
    RawPool<BatchDecoder>::put(BD(decoder));
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_add_original(SgpuDecoder decoder, unsigned packetNum,
                                                       const void* deviceData, unsigned bytes)
{
    if (!decoder || BD(decoder)->core.ge_pending() || !deviceData || bytes == 0 || bytes > SIAMESE_MAX_PACKET_BYTES ||
        packetNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    SiameseOriginalPacket p;
    p.PacketNum = packetNum;
    p.Data = (const unsigned char*)deviceData;
    p.DataBytes = bytes;
    return BD(decoder)->core.add_original(p, (uint64_t)(uintptr_t)deviceData);
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_add_original_range(SgpuDecoder decoder, unsigned firstPacketNum,
                                                             const void* deviceData, size_t stride,
                                                             const unsigned* bytes, unsigned fixedBytes,
                                                             unsigned count, SiameseResult* results,
                                                             unsigned* callsOut)
{
    if (callsOut)
        *callsOut = 0;
    if (!decoder || BD(decoder)->core.ge_pending() || (!deviceData && count) || firstPacketNum > SIAMESE_PACKET_NUM_MAX || stride > 0xffffffffu ||
        (count > 1 && stride == 0))
        return Siamese_InvalidInput;
    unsigned calls = 0;
    const SiameseResult r = BD(decoder)->core.add_original_range(firstPacketNum, (uint64_t)(uintptr_t)deviceData,
                                                                 (uint32_t)stride, bytes, fixedBytes, count, results,
                                                                 &calls);
    if (callsOut)
        *callsOut = calls;
    return r;
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_add_recovery(SgpuDecoder decoder, const SgpuRecoveryPacket* packet)
{
    if (!decoder || BD(decoder)->core.ge_pending() || !packet || !packet->DeviceData || packet->DataBytes == 0 ||
        packet->FooterBytes == 0 || packet->FooterBytes > 8 || packet->FooterBytes >= packet->DataBytes)
        return Siamese_InvalidInput;
    DeviceRecovery r;
    r.data = (uint64_t)(uintptr_t)packet->DeviceData;
    r.bytes = packet->DataBytes;
    r.footer = packet->Footer;
    r.footerBytes = packet->FooterBytes;
    r.head = packet->Head;
    r.producer = reinterpret_cast<Program*>(packet->Producer);
    return BD(decoder)->core.add_recovery_device(r);
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_is_ready(SgpuDecoder decoder)
{
    if (!decoder || BD(decoder)->core.ge_pending())
        return Siamese_InvalidInput;
    return BD(decoder)->core.is_ready();
}

SIAMESE_EXPORT SiameseResult sgpu_decode(SgpuDecoder decoder, SiameseOriginalPacket** packetsOut,
                                         unsigned* countOut)
{
    if (!decoder || BD(decoder)->core.ge_pending() || (!packetsOut != !countOut))
        return Siamese_InvalidInput;
    return BD(decoder)->core.decode(packetsOut, countOut);
}

SIAMESE_EXPORT SiameseResult sgpu_decode_device(SgpuDecoder decoder, SiameseOriginalPacket** packetsOut,
                                                unsigned* countOut)
{
    if (!decoder || (!packetsOut != !countOut))
        return Siamese_InvalidInput;
    return BD(decoder)->core.decode_device(packetsOut, countOut);
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_get(SgpuDecoder decoder, SiameseOriginalPacket* packet)
{
    if (!decoder || BD(decoder)->core.ge_pending() || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    return BD(decoder)->core.get(*packet);
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_get_range(SgpuDecoder decoder, unsigned firstPacketNum, unsigned count,
                                                    SiameseOriginalPacket* packets, unsigned* gotOut)
{
    if (gotOut)
        *gotOut = 0;
    if (!decoder || BD(decoder)->core.ge_pending() || (!packets && count) || !gotOut || firstPacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    return BD(decoder)->core.get_range(firstPacketNum, count, packets, gotOut);
}

SIAMESE_EXPORT SiameseResult sgpu_decode_deferred(SgpuDecoder decoder, SiameseOriginalPacket* out,
                                                  unsigned capacity, unsigned* countOut)
{
    if (!decoder || BD(decoder)->core.ge_pending() || !out || !countOut)
        return Siamese_InvalidInput;
    return BD(decoder)->core.decode_deferred(out, capacity, countOut);
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_get_deferred(SgpuDecoder decoder, SiameseOriginalPacket* packet)
{
    if (!decoder || BD(decoder)->core.ge_pending() || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    return BD(decoder)->core.get_deferred(*packet);
}

SIAMESE_EXPORT SiameseResult sgpu_decoder_has(SgpuDecoder decoder, unsigned packetNum)
{
    if (!decoder || BD(decoder)->core.ge_pending() || packetNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    return BD(decoder)->core.has(packetNum) ? Siamese_Success : Siamese_NeedMoreData;
}

SIAMESE_EXPORT int sgpu_flush(void)
{
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    return eng->flush_and_sync() ? 0 : -1;
}

SIAMESE_EXPORT int sgpu_submit(void)
{
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    return eng->flush() ? 0 : -1;
}

SIAMESE_EXPORT long long sgpu_enqueue(void)
{
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    const uint64_t t = eng->enqueue();
    return eng->failed() ? -1 : (long long)t;
}

SIAMESE_EXPORT int sgpu_wait(long long ticket)
{
    // no engine lock: other threads keep driving instances meanwhile
    if (ticket < 0)
        return -1;
    return Engine::global()->wait((uint64_t)ticket) ? 0 : -1;
}

SIAMESE_EXPORT int sgpu_query(long long ticket)
{
    Engine* eng = Engine::global();
    if (ticket < 0 || eng->failed())
        return -1;
    return eng->done((uint64_t)ticket) ? 1 : 0;
}

SIAMESE_EXPORT void sgpu_parallel_for(unsigned count, void (*fn)(void* ctx, unsigned index), void* ctx)
{
    if (!fn)
        return;
    Engine::global()->pool().run(count, [&](size_t i) { fn(ctx, (unsigned)i); });
}

SIAMESE_EXPORT void* sgpu_device_alloc(size_t bytes)
{
    if (!g_batchReady)
        return nullptr;
    Lock lock(Engine::global()->mutex());
    return be_dev_alloc(bytes);
}

SIAMESE_EXPORT void sgpu_device_free(void* p)
{
    Lock lock(Engine::global()->mutex());
    be_dev_free(p);
}

SIAMESE_EXPORT void* sgpu_host_alloc(size_t bytes)
{
    if (!g_batchReady)
        return nullptr;
    Lock lock(Engine::global()->mutex());
    return be_host_alloc(bytes);
}

SIAMESE_EXPORT void sgpu_host_free(void* p)
{
    Lock lock(Engine::global()->mutex());
    be_host_free(p);
}

SIAMESE_EXPORT int sgpu_h2d(void* deviceDst, const void* hostSrc, size_t bytes)
{
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    if (!eng->sync())
        return -1;
    be_h2d(deviceDst, hostSrc, bytes);
    return be_sync() ? 0 : -1;
}

SIAMESE_EXPORT int sgpu_gather(unsigned count, const void* const* deviceSrcs, const unsigned* bytes,
                               void* hostOut)
{
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    return eng->gather(count, deviceSrcs, bytes, hostOut) ? 0 : -1;
}

SIAMESE_EXPORT int sgpu_h2d_async(void* deviceDst, const void* hostSrc, size_t bytes)
{
    if (!g_batchReady)
        return -1;
    return Engine::global()->stage_in(deviceDst, hostSrc, bytes) ? 0 : -1;
}

SIAMESE_EXPORT int sgpu_gather_completed(unsigned count, const void* const* deviceSrcs, const unsigned* bytes,
                                         void* pinnedOut)
{
    if (!g_batchReady)
        return -1;
    return Engine::global()->gather_completed(count, deviceSrcs, bytes, pinnedOut) ? 0 : -1;
}

SIAMESE_EXPORT long long sgpu_gather_async(unsigned count, const void* const* deviceSrcs, const unsigned* bytes,
                                           void* pinnedOut)
{
    if (!g_batchReady)
        return -1;
    return (long long)Engine::global()->gather_async(count, deviceSrcs, bytes, pinnedOut);
}

SIAMESE_EXPORT int sgpu_gather_wait(long long ticket)
{
    if (!g_batchReady)
        return -1;
    return Engine::global()->gather_wait((int64_t)ticket) ? 0 : -1;
}

SIAMESE_EXPORT unsigned sgpu_frame_header_bytes(unsigned type, unsigned dataBytes)
{
    if (type > SGPU_FRAME_RECOVERY)
        return 0;
    return frame_header_bytes(type, dataBytes);
}

SIAMESE_EXPORT unsigned sgpu_frame_write_header(unsigned type, unsigned flow, unsigned packetNum,
                                                unsigned dataBytes, void* out)
{
    if (!out || type > SGPU_FRAME_RECOVERY || flow > kFrameMaxFlow || packetNum > SIAMESE_PACKET_NUM_MAX ||
        dataBytes == 0 || dataBytes > SIAMESE_MAX_PACKET_BYTES)
        return 0;
    return frame_write_header(type, flow, packetNum, dataBytes, static_cast<uint8_t*>(out));
}

SIAMESE_EXPORT SiameseResult sgpu_frames_parse(const void* frames, size_t bytes, SgpuFrame* out,
                                               unsigned maxFrames, unsigned* countOut)
{
    if (!frames || !out || !countOut)
        return Siamese_InvalidInput;
    *countOut = 0;
    if (bytes > UINT32_MAX)   // (frame offsets are 32-bit)
        return Siamese_InvalidInput;
    static_assert(sizeof(SgpuFrame) == sizeof(FrameInfo), "SgpuFrame layout");
    size_t consumed = 0, bad = 0;
    const long n = frames_parse(static_cast<const uint8_t*>(frames), bytes, reinterpret_cast<FrameInfo*>(out),
                                maxFrames, &consumed, &bad);
    // (the frames before a malformed one are returned with InvalidInput)
    *countOut = (unsigned)n;
    return consumed == bytes && bad == kNoBadFrame ? Siamese_Success : Siamese_InvalidInput;
}

SIAMESE_EXPORT SiameseResult sgpu_frames_recv(const SgpuDecoder* decoders, unsigned decoderCount,
                                              const void* hostFrames, const void* deviceFrames, size_t bytes,
                                              SiameseResult* results, unsigned maxFrames, unsigned* countOut)
{
    if (!decoders || !hostFrames || !deviceFrames || !countOut)
        return Siamese_InvalidInput;
    *countOut = 0;
    if (bytes > UINT32_MAX)   // (frame offsets are 32-bit)
        return Siamese_InvalidInput;
    const uint8_t* host = static_cast<const uint8_t*>(hostFrames);
    const uint64_t dev = (uint64_t)(uintptr_t)deviceFrames;
    // parse in blocks: the headers of a whole ring in one pass, then the calls
    FrameInfo fi[256];
    size_t at = 0;
    unsigned done = 0;
    SiameseResult status = Siamese_Success;
    bool malformed = false;
    while (at < bytes && done < maxFrames && !malformed) {
        size_t consumed = 0, bad = 0;
        const size_t want = std::min<size_t>(256, maxFrames - done);
        const long n = frames_parse(host + at, bytes - at, fi, want, &consumed, &bad);
        // every well-formed frame before a malformed one is still delivered;
        // the ring is not read past the malformed frame (its length cannot be
        // trusted to find the next one)
        malformed = bad != kNoBadFrame;
        for (long k = 0; k < n; ++k) {
            const FrameInfo& f = fi[k];
            const size_t off = at + f.offset;
            SiameseResult r = Siamese_InvalidInput;
            SgpuDecoder d = f.flow < decoderCount ? decoders[f.flow] : nullptr;
            // (a decoder with a device matrix job in flight takes no packets:
            // the job was built from its current window, like every other
            // sgpu_decoder_* call it answers InvalidInput until decode_device
            // has finished the job)
            if (d && BD(d)->core.ge_pending())
                d = nullptr;
            if (d && f.type == kFrameOriginal) {
                if (f.bytes <= SIAMESE_MAX_PACKET_BYTES && f.packetNum <= SIAMESE_PACKET_NUM_MAX) {
                    SiameseOriginalPacket p;
                    p.PacketNum = f.packetNum;
                    p.Data = reinterpret_cast<const unsigned char*>((uintptr_t)(dev + off));
                    p.DataBytes = f.bytes;
                    r = BD(d)->core.add_original(p, dev + off);
                }
            } else if (d && f.type == kFrameRecovery) {
                RowMeta m;
                const int footer = read_footer(host + off, f.bytes, &m);
                if (footer > 0 && (unsigned)footer < f.bytes) {
                    DeviceRecovery rec;
                    rec.data = dev + off;
                    rec.bytes = f.bytes;
                    rec.footer = host + off + f.bytes - footer;
                    rec.footerBytes = (unsigned)footer;
                    rec.head = host + off;
                    rec.producer = nullptr;   // staged: ingested from the device copy
                    r = BD(d)->core.add_recovery_device(rec);
                }
            }
            if (results)
                results[done] = r;
            if (r != Siamese_Success && status == Siamese_Success)
                status = r;
            ++done;
        }
        at += consumed;
        if (n == 0)
            break;
    }
    *countOut = done;
    return at >= bytes && !malformed ? status : Siamese_InvalidInput;
}

SIAMESE_EXPORT long long sgpu_frames_send(unsigned count, const SgpuRecoveryPacket* packets, const unsigned* flows,
                                          void* pinnedOut, size_t capacity, size_t* bytesOut)
{
    if (!g_batchReady || !packets || !flows || !pinnedOut || !bytesOut)
        return -1;
    std::vector<const void*> srcs(count);
    std::vector<unsigned> lens(count), hlen(count);
    std::vector<uint8_t> hdr((size_t)count * 8);
    size_t total = 0;
    for (unsigned i = 0; i < count; ++i) {
        // (as sgpu_frame_write_header: an empty or oversized packet is no frame)
        if (!packets[i].DeviceData || flows[i] > kFrameMaxFlow || packets[i].DataBytes == 0 ||
            packets[i].DataBytes > SIAMESE_MAX_PACKET_BYTES)
            return -1;
        srcs[i] = packets[i].DeviceData;
        lens[i] = packets[i].DataBytes;
        hlen[i] = frame_write_header(kFrameRecovery, flows[i], 0, lens[i], hdr.data() + 8 * (size_t)i);
        if (hlen[i] > 8)
            return -1;
        total = (total + hlen[i] + lens[i] + 15) & ~(size_t)15;
    }
    *bytesOut = total;
    if (total > capacity)
        return -1;
    return (long long)Engine::global()->gather_async_framed(count, srcs.data(), lens.data(), hdr.data(), hlen.data(),
                                                            pinnedOut);
}

SIAMESE_EXPORT void sgpu_timing(int enable, int reset, double* execMs, double* totalMs)
{
    be_timing_enable(enable != 0);
    if (execMs)
        *execMs = be_timing_exec_ms();
    if (totalMs)
        *totalMs = be_timing_total_ms();
    if (reset)
        be_timing_reset();
}

SIAMESE_EXPORT void sgpu_timing_kernels(double* msOut, unsigned count)
{
    for (unsigned k = 0; k < count && k < kBeKernelKinds; ++k)
        msOut[k] = be_timing_kernel_ms((BeKernel)k);
}

SIAMESE_EXPORT void sgpu_engine_stats_ex(uint64_t* out, unsigned count)
{
    const EngineStats s = Engine::global()->stats();
    const uint64_t v[20] = {s.flushes,    s.launches,    s.ops,        s.terms,    s.solves,
                            s.ingests,    s.uploadBytes, s.refOpBytes, s.outBytes, s.solveBytes,
                            s.assembleNs, s.waitNs,      s.completeNs, s.reclaimNs,
                            s.execLaunches, s.ldpcBytes, s.execUniqueBytes,
                            s.geJobs,     s.geChained,   s.geRetried};
    for (unsigned k = 0; k < count && k < 20; ++k)
        out[k] = v[k];
}

SIAMESE_EXPORT void sgpu_measure_unique(int on)
{
    Engine::set_measure_unique(on != 0);
}

SIAMESE_EXPORT void sgpu_engine_stats(uint64_t* out15)
{
    const EngineStats s = Engine::global()->stats();
    const uint64_t v[15] = {s.flushes,    s.launches,    s.ops,        s.terms,    s.solves,
                            s.ingests,    s.uploadBytes, s.refOpBytes, s.outBytes, s.solveBytes,
                            s.assembleNs, s.waitNs,      s.completeNs, s.reclaimNs,
                            s.execLaunches};
    std::memcpy(out15, v, sizeof(v));
}

SIAMESE_EXPORT uint64_t sgpu_arena_bytes(void)
{
    return Engine::global()->arena_bytes();
}

SIAMESE_EXPORT int sgpu_arena_reserve(size_t bytes)
{
    if (!g_batchReady)
        return -1;
    return Engine::global()->reserve(bytes) ? 0 : -1;
}

} // extern "C"
