/*
    siamese.h -- drop-in C ABI of the MI355X streaming erasure codec.

    Every declaration below keeps the exact name, signature, enum value and
    struct layout of the upstream interface (reference: siamese.h:91-583), so
    an application (or an FFI stub generated from the upstream header) links
    against libsiamese_amd.so unchanged.  What differs is the machinery behind
    it: symbol arithmetic runs as HIP kernels on an MI355X, the control plane
    stays on the host.

    Reference interface replaced, per entry point:
      siamese_init_                  siamese.h:128   (siamese.cpp:43-53)
      siamese_encoder_create/free    siamese.h:213/216 (siamese.cpp:58-74)
      siamese_encoder_is_ready       siamese.h:231   (siamese.cpp:76-94)
      siamese_encoder_add            siamese.h:250   (siamese.cpp:96-108)
      siamese_encoder_get            siamese.h:263   (siamese.cpp:110-121)
      siamese_encoder_remove_before  siamese.h:278   (siamese.cpp:123-133)
      siamese_encoder_ack            siamese.h:299   (siamese.cpp:135-146)
      siamese_encoder_retransmit     siamese.h:326   (siamese.cpp:148-157)
      siamese_encode                 siamese.h:349   (siamese.cpp:159-168)
      siamese_decoder_create/free    siamese.h:366/369 (siamese.cpp:186-205)
      siamese_decoder_add_original   siamese.h:380   (siamese.cpp:207-220)
      siamese_decoder_add_recovery   siamese.h:397   (siamese.cpp:222-234)
      siamese_decoder_get            siamese.h:416   (siamese.cpp:236-245)
      siamese_decoder_is_ready       siamese.h:426   (siamese.cpp:247-255)
      siamese_decode                 siamese.h:453   (siamese.cpp:257-269)
      siamese_decoder_ack            siamese.h:478   (siamese.cpp:271-286)
      siamese_encoder_stats          siamese.h:527   (siamese.cpp:170-180)
      siamese_decoder_stats          siamese.h:579   (siamese.cpp:288-299)
*/
#ifndef CAT_SIAMESE_H
#define CAT_SIAMESE_H

#define SIAMESE_VERSION 5

#if defined(SIAMESE_BUILDING)
# define SIAMESE_EXPORT __attribute__((visibility("default")))
#else
# define SIAMESE_EXPORT extern
#endif

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Initialization ---------------------------------------------------- */

/* Returns 0 on success.  Also binds the calling process to the HIP device
   selected by SIAMESE_AMD_DEVICE (default: the current HIP device). */
SIAMESE_EXPORT int siamese_init_(int version);
#define siamese_init() siamese_init_(SIAMESE_VERSION)

/* ---- Shared constants and types ---------------------------------------- */

typedef enum SiameseResultT
{
    Siamese_Success           = 0,
    Siamese_InvalidInput      = 1,
    Siamese_NeedMoreData      = 2,
    Siamese_MaxPacketsReached = 3,
    Siamese_DuplicateData     = 4,
    Siamese_Disabled          = 5,   /* sticky: codec refused further work */

    SiameseResult_Count,
    SiameseResult_Padding = 0x7fffffff
} SiameseResult;

#define SIAMESE_RECOVERY_NUM_MIN         0
#define SIAMESE_RECOVERY_NUM_MAX       255
#define SIAMESE_RECOVERY_NUM_COUNT     256

#define SIAMESE_MAX_PACKETS          16000

#define SIAMESE_PACKET_NUM_MIN           0
#define SIAMESE_PACKET_NUM_MAX    0x3fffff
#define SIAMESE_PACKET_NUM_COUNT  0x400000
#define SIAMESE_PACKET_NUM_BITS         22
#define SIAMESE_PACKET_NUM_INC(x)  ( (x + 1) & (SIAMESE_PACKET_NUM_COUNT - 1) )

#define SIAMESE_MIN_PACKET_BYTES         1
#define SIAMESE_MAX_PACKET_BYTES 536870911 /* 0x1fffffff */

#define SIAMESE_MAX_ENCODE_OVERHEAD     8
#define SIAMESE_ACK_MIN_BYTES          16

struct SiameseOriginalPacket
{
    unsigned PacketNum;
    unsigned DataBytes;
    const unsigned char* Data;
};

struct SiameseRecoveryPacket
{
    unsigned DataBytes;
    const unsigned char* Data;
};

/* ---- Encoder ------------------------------------------------------------ */

typedef struct SiameseEncoderImpl { int impl; }* SiameseEncoder;

SIAMESE_EXPORT SiameseEncoder siamese_encoder_create();
SIAMESE_EXPORT void siamese_encoder_free(SiameseEncoder encoder);
SIAMESE_EXPORT SiameseResult siamese_encoder_is_ready(SiameseEncoder encoder);
SIAMESE_EXPORT SiameseResult siamese_encoder_add(SiameseEncoder encoder,
                                                 SiameseOriginalPacket* packet);
SIAMESE_EXPORT SiameseResult siamese_encoder_get(SiameseEncoder encoder,
                                                 SiameseOriginalPacket* packet);
SIAMESE_EXPORT SiameseResult siamese_encoder_remove_before(SiameseEncoder encoder,
                                                           unsigned firstKeptPacketNum);
SIAMESE_EXPORT SiameseResult siamese_encoder_ack(SiameseEncoder encoder,
                                                 const void* buffer, unsigned bytes,
                                                 unsigned* nextExpectedPacketNum);
SIAMESE_EXPORT SiameseResult siamese_encoder_retransmit(SiameseEncoder encoder,
                                                        SiameseOriginalPacket* original);
/* The returned Data stays valid until the next siamese_encode() call. */
SIAMESE_EXPORT SiameseResult siamese_encode(SiameseEncoder encoder,
                                            SiameseRecoveryPacket* recovery);

/* ---- Decoder ------------------------------------------------------------ */

typedef struct SiameseDecoderImpl { int impl; }* SiameseDecoder;

SIAMESE_EXPORT SiameseDecoder siamese_decoder_create();
SIAMESE_EXPORT void siamese_decoder_free(SiameseDecoder decoder);
SIAMESE_EXPORT SiameseResult siamese_decoder_add_original(SiameseDecoder decoder,
                                                          const SiameseOriginalPacket* packet);
SIAMESE_EXPORT SiameseResult siamese_decoder_add_recovery(SiameseDecoder decoder,
                                                          const SiameseRecoveryPacket* packet);
/* Returned Data valid until add_recovery / decode / free. */
SIAMESE_EXPORT SiameseResult siamese_decoder_get(SiameseDecoder decoder,
                                                 SiameseOriginalPacket* packet);
SIAMESE_EXPORT SiameseResult siamese_decoder_is_ready(SiameseDecoder decoder);
/* Output array is in increasing PacketNum order; valid until add_recovery /
   decode / free. */
SIAMESE_EXPORT SiameseResult siamese_decode(SiameseDecoder decoder,
                                            SiameseOriginalPacket** packetsPtrOut,
                                            unsigned* countOut);
SIAMESE_EXPORT SiameseResult siamese_decoder_ack(SiameseDecoder decoder,
                                                 void* buffer, unsigned byteLimit,
                                                 unsigned* usedBytes);

/* ---- Statistics ----------------------------------------------------------- */

typedef enum SiameseEncoderStatsT
{
    SiameseEncoderStats_OriginalCount,
    SiameseEncoderStats_OriginalBytes,
    SiameseEncoderStats_RecoveryCount,
    SiameseEncoderStats_RecoveryBytes,
    SiameseEncoderStats_RetransmitCount,
    SiameseEncoderStats_RetransmitBytes,
    SiameseEncoderStats_AckCount,
    SiameseEncoderStats_AckBytes,
    SiameseEncoderStats_MemoryUsed,
    SiameseEncoderStats_Count
} SiameseEncoderStats;

SIAMESE_EXPORT SiameseResult siamese_encoder_stats(SiameseEncoder encoder,
                                                   uint64_t* statsOut, unsigned statsCount);

typedef enum SiameseDecoderStatsT
{
    SiameseDecoderStats_OriginalCount,
    SiameseDecoderStats_OriginalBytes,
    SiameseDecoderStats_RecoveryCount,
    SiameseDecoderStats_RecoveryBytes,
    SiameseDecoderStats_AckCount,
    SiameseDecoderStats_AckBytes,
    SiameseDecoderStats_DupedOriginalCount,
    SiameseDecoderStats_SolveSuccessCount,
    SiameseDecoderStats_SolveFailCount,
    SiameseDecoderStats_DupedRecoveryCount,
    SiameseDecoderStats_MemoryUsed,
    SiameseDecoderStats_Count
} SiameseDecoderStats;

SIAMESE_EXPORT SiameseResult siamese_decoder_stats(SiameseDecoder decoder,
                                                   uint64_t* statsOut, unsigned statsCount);

#ifdef __cplusplus
}
#endif

#endif /* CAT_SIAMESE_H */
