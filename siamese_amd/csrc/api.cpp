// api.cpp -- the drop-in siamese.h entry points (reference siamese.cpp:35-302).
//
// Argument validation and result codes follow the reference entry points
// one-for-one.  The reference API is not thread-safe (siamese.h:59: "a lock
// should be held while calling").  This library keeps that contract for one
// instance and extends it: calls on different instances may run concurrently,
// holding the engine's instance lock shared.  Calls that
// must hand host memory back to the caller (siamese_encode, siamese_decode,
// and siamese_decoder_get on a freshly recovered packet) queue their device
// work, drop the lock and flush: concurrent flushes commit as a group (the
// first carries everything queued before it, Engine::flush_and_sync), and no
// thread holds a lock across a device round trip.  The bytes land in host
// buffers whose lifetime matches the reference contract (siamese.h:335-336,
// :410-414).
#define SIAMESE_BUILDING
#include "../../include/siamese.h"

#include "backend.h"
#include "decoder.h"
#include "encoder.h"
#include "engine.h"

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <new>
#include <shared_mutex>

using namespace sgpu;

namespace {

bool g_initialized = false;

struct ApiEncoder
{
    EncoderCore core{Engine::global(), true};
    std::vector<uint8_t> out; // last recovery packet (host copy)
};

struct ApiDecoder
{
    DecoderCore core{Engine::global(), true};
};

inline ApiEncoder* E(SiameseEncoder e) { return reinterpret_cast<ApiEncoder*>(e); }
inline ApiDecoder* D(SiameseDecoder d) { return reinterpret_cast<ApiDecoder*>(d); }

using Lock = std::lock_guard<std::mutex>;
// an instance call (shared: other instances' calls run beside it)
struct Shared
{
    std::shared_lock<InstanceLock> l;
    Shared() : l(Engine::global()->instance_lock()) {}
};

} // namespace

extern "C" {

SIAMESE_EXPORT int siamese_init_(int version)
{
    if (version != SIAMESE_VERSION)
        return Siamese_Disabled;
    if (!gf_init())
        return Siamese_Disabled;
    Engine* eng = Engine::global();
    Lock lock(eng->mutex());
    const char* err = "unknown";
    int device = -1;
    if (const char* s = std::getenv("SIAMESE_AMD_DEVICE"))
        device = std::atoi(s);
    if (!eng->init(device, &err)) {
        std::fprintf(stderr, "siamese_amd: initialisation failed: %s\n", err);
        return Siamese_Disabled;
    }
    g_initialized = true;
    return Siamese_Success;
}

// ---- Encoder --------------------------------------------------------------

SIAMESE_EXPORT SiameseEncoder siamese_encoder_create()
{
    if (!g_initialized)
        return nullptr;
    Shared lock;
    return reinterpret_cast<SiameseEncoder>(new (std::nothrow) ApiEncoder);
}

SIAMESE_EXPORT void siamese_encoder_free(SiameseEncoder encoder)
{
    if (!encoder)
        return;
    Shared lock;
    delete E(encoder);
}

SIAMESE_EXPORT SiameseResult siamese_encoder_is_ready(SiameseEncoder encoder)
{
    if (!encoder)
        return Siamese_InvalidInput;
    Shared lock;
    // keep two slots of slack for the application (siamese.cpp:86-91)
    if (E(encoder)->core.remaining_slots() <= 2)
        return Siamese_MaxPacketsReached;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_add(SiameseEncoder encoder, SiameseOriginalPacket* packet)
{
    if (!encoder || !packet || !packet->Data || packet->DataBytes <= 0 ||
        packet->DataBytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    Shared lock;
    return E(encoder)->core.add(*packet);
}

SIAMESE_EXPORT SiameseResult siamese_encoder_get(SiameseEncoder encoder, SiameseOriginalPacket* packet)
{
    if (!encoder || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    Shared lock;
    return E(encoder)->core.get(*packet);
}

SIAMESE_EXPORT SiameseResult siamese_encoder_remove_before(SiameseEncoder encoder, unsigned packetNum)
{
    if (!encoder || packetNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    Shared lock;
    E(encoder)->core.remove_before(packetNum);
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_ack(SiameseEncoder encoder, const void* buffer,
                                                 unsigned bytes, unsigned* nextExpectedPacketNum)
{
    if (!encoder || !buffer || bytes < 1 || !nextExpectedPacketNum)
        return Siamese_InvalidInput;
    Shared lock;
    return E(encoder)->core.acknowledge((const uint8_t*)buffer, bytes, *nextExpectedPacketNum);
}

SIAMESE_EXPORT SiameseResult siamese_encoder_retransmit(SiameseEncoder encoder,
                                                        SiameseOriginalPacket* original)
{
    if (!encoder || !original)
        return Siamese_InvalidInput;
    Shared lock;
    return E(encoder)->core.retransmit(*original);
}

SIAMESE_EXPORT SiameseResult siamese_encode(SiameseEncoder encoder, SiameseRecoveryPacket* recovery)
{
    if (!encoder || !recovery)
        return Siamese_InvalidInput;
    Engine* eng = Engine::global();
    ApiEncoder* enc = E(encoder);
    EncodeOut o;
    {
        Shared lock;
        const SiameseResult r = enc->core.encode(o);
        if (r != Siamese_Success) {
            if (r == Siamese_NeedMoreData)
                recovery->DataBytes = 0;
            return r;
        }
        enc->out.resize(o.bytes);
        eng->download(enc->out.data(), o.buf.addr(), o.bytes);
    }
    if (!eng->flush_and_sync(&eng->instance_lock()))
        return Siamese_Disabled;
    recovery->Data = enc->out.data();
    recovery->DataBytes = o.bytes;
    return Siamese_Success;
}

SIAMESE_EXPORT SiameseResult siamese_encoder_stats(SiameseEncoder encoder, uint64_t* statsOut,
                                                   unsigned statsCount)
{
    if (!encoder || !statsOut || statsCount <= 0)
        return Siamese_InvalidInput;
    Shared lock;
    return E(encoder)->core.stats(statsOut, statsCount);
}

// ---- Decoder --------------------------------------------------------------

SIAMESE_EXPORT SiameseDecoder siamese_decoder_create()
{
    if (!g_initialized)
        return nullptr;
    Shared lock;
    return reinterpret_cast<SiameseDecoder>(new (std::nothrow) ApiDecoder);
}

SIAMESE_EXPORT void siamese_decoder_free(SiameseDecoder decoder)
{
    if (!decoder)
        return;
    Shared lock;
    delete D(decoder);
}

SIAMESE_EXPORT SiameseResult siamese_decoder_add_original(SiameseDecoder decoder,
                                                          const SiameseOriginalPacket* packet)
{
    if (!decoder || !packet || packet->DataBytes <= 0 || packet->DataBytes > SIAMESE_MAX_PACKET_BYTES ||
        packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    Shared lock;
    return D(decoder)->core.add_original(*packet);
}

SIAMESE_EXPORT SiameseResult siamese_decoder_add_recovery(SiameseDecoder decoder,
                                                          const SiameseRecoveryPacket* packet)
{
    if (!decoder || !packet || !packet->Data || packet->DataBytes <= 0 ||
        packet->DataBytes > SIAMESE_MAX_PACKET_BYTES)
        return Siamese_InvalidInput;
    Shared lock;
    return D(decoder)->core.add_recovery(*packet);
}

SIAMESE_EXPORT SiameseResult siamese_decoder_get(SiameseDecoder decoder, SiameseOriginalPacket* packet)
{
    if (!decoder || !packet || packet->PacketNum > SIAMESE_PACKET_NUM_MAX)
        return Siamese_InvalidInput;
    Engine* eng = Engine::global();
    DecoderCore& core = D(decoder)->core;
    {
        Shared lock;
        const SiameseResult r = core.get(*packet);
        if (r != kNeedsFlush)
            return r;
    }
    // a freshly recovered packet whose exact length is still on the device:
    // flushed outside the instance lock (DecoderCore::get never flushes in
    // drop-in mode, so no thread waits for the lock's exclusive side while
    // holding its shared side)
    if (!eng->flush_and_sync(&eng->instance_lock()))
        return Siamese_Disabled;
    Shared lock;
    const SiameseResult r = core.get(*packet);
    return r == kNeedsFlush ? Siamese_Disabled : r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_is_ready(SiameseDecoder decoder)
{
    if (!decoder)
        return Siamese_InvalidInput;
    Shared lock;
    return D(decoder)->core.is_ready();
}

SIAMESE_EXPORT SiameseResult siamese_decode(SiameseDecoder decoder, SiameseOriginalPacket** packetsPtrOut,
                                            unsigned* countOut)
{
    if (!decoder || (!packetsPtrOut != !countOut))
        return Siamese_InvalidInput;
    Engine* eng = Engine::global();
    DecoderCore& core = D(decoder)->core;
    SiameseResult r;
    {
        Shared lock;
        r = core.decode(packetsPtrOut, countOut);
        if (!core.has_pending())
            return r;
        core.download_recovered();
    }
    if (!eng->flush_and_sync(&eng->instance_lock()))
        return Siamese_Disabled;
    Shared lock;
    if (core.disabled())   // (applies the completed solve first)
        return Siamese_Disabled;
    return r;
}

SIAMESE_EXPORT SiameseResult siamese_decoder_ack(SiameseDecoder decoder, void* buffer, unsigned byteLimit,
                                                 unsigned* usedBytes)
{
    if (!decoder || !buffer || !usedBytes || byteLimit < SIAMESE_ACK_MIN_BYTES)
        return Siamese_InvalidInput;
    Shared lock;
    return D(decoder)->core.acknowledgement((uint8_t*)buffer, byteLimit, *usedBytes);
}

SIAMESE_EXPORT SiameseResult siamese_decoder_stats(SiameseDecoder decoder, uint64_t* statsOut,
                                                   unsigned statsCount)
{
    if (!decoder || !statsOut || statsCount <= 0)
        return Siamese_InvalidInput;
    Shared lock;
    return D(decoder)->core.stats(statsOut, statsCount);
}

} // extern "C"
