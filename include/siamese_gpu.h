/*
    siamese_gpu.h -- device-resident batch API of libsiamese_amd (additive;
    not part of the upstream interface).

    siamese.h moves every packet through host memory and waits for the GPU on
    each siamese_encode / siamese_decode, which is the drop-in contract.  This
    header exposes the same codec with packets that stay in HBM:

      * originals are ingested from device pointers;
      * siamese_encode's result is a device-resident recovery packet that can
        be handed straight to a decoder on the same GPU;
      * nothing waits for the GPU until sgpu_flush(), so thousands of
        independent encoder/decoder pairs are driven per kernel launch.

    Per-instance call semantics, result codes and outputs are those of the
    corresponding siamese.h call (reference siamese.h:213-483); only the data
    location and the completion point differ.  Recovered packets returned by
    sgpu_decode carry device pointers whose DataBytes are exact after the
    next sgpu_flush() (they read 0 until then).

    Device pointer lifetime: a symbol an instance drops (a decoder sliding its
    window past delivered packets, a freed instance) is recycled once the
    submission holding that call has completed, and any later submission may
    then rewrite it.  Read (sgpu_gather_async / sgpu_gather_completed) the
    bytes behind a pointer from sgpu_decode, sgpu_decoder_get or sgpu_encode
    after the submission that produced them completes and before the next
    submission is enqueued; the gather's reads are ordered before that
    submission's device work.

    Threading: instances may be driven from many host threads at once, each
    instance by one thread at a time (handing a recovery packet to a decoder
    also touches the encoder that produced it).  Per-instance calls take no
    global lock.  sgpu_init, sgpu_flush, sgpu_submit, sgpu_enqueue,
    sgpu_gather, sgpu_h2d, and sgpu_decoder_get on a packet whose length is
    still pending (it flushes) must not run concurrently with any other call;
    sgpu_h2d_async and sgpu_gather_completed may run beside instance calls.

    Pipelined submission: sgpu_enqueue() hands all queued work to the
    library's launcher thread and returns a ticket at once; sgpu_wait(ticket)
    returns when that submission (and every earlier one) has run on the GPU
    and its results are delivered.  sgpu_wait may run while other threads
    drive instances.  An instance may be driven on while its earlier
    submissions are still in flight (a single stream keeps the GPU busy with
    one submission while the host prepares the next): completions never
    touch an instance's state behind its back, each call first applies the
    completions that have arrived.

    Deferred outputs: sgpu_decode_deferred and sgpu_decoder_get_deferred
    never wait for the GPU.  They write into entries the caller owns; an
    entry whose packet is still being solved gets its Data and DataBytes
    when the submission carrying the solve completes, before sgpu_query /
    sgpu_wait report that submission (or a later one) done.  The caller keeps
    such entries alive until then (freeing the decoder does not cancel them).
*/
#ifndef SIAMESE_GPU_H
#define SIAMESE_GPU_H

#include "siamese.h"
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct SgpuEncoderImpl { int impl; }* SgpuEncoder;
typedef struct SgpuDecoderImpl { int impl; }* SgpuDecoder;

/// Device-resident recovery packet (valid until the next sgpu_encode on the
/// same encoder).  Footer/Head are host copies the decoder parses directly.
typedef struct SgpuRecoveryPacket
{
    const unsigned char* DeviceData;   ///< payload + footer in HBM
    unsigned DataBytes;
    unsigned FooterBytes;
    unsigned char Footer[8];
    unsigned char Head[4];
    void* Producer;                    ///< internal: encoder that owns DeviceData
} SgpuRecoveryPacket;

/// Initialise the library on HIP device `device` (<0: current device).
SIAMESE_EXPORT int sgpu_init(int device);

SIAMESE_EXPORT SgpuEncoder sgpu_encoder_create(void);
SIAMESE_EXPORT void sgpu_encoder_free(SgpuEncoder encoder);
SIAMESE_EXPORT SiameseResult sgpu_encoder_add(SgpuEncoder encoder, const void* deviceData,
                                              unsigned bytes, unsigned* packetNumOut);
/// `count` sgpu_encoder_add calls in one: original k's payload at
/// deviceData + k * stride, bytes[k] bytes (fixedBytes for all when bytes is
/// NULL).  Identical to the calls made in order until one fails, whose
/// result is returned (Success if none did); *addedOut = originals added,
/// the first as packet *firstPacketNumOut and the others after it.  The
/// originals of one subwindow fill one slab: a run of adds costs one
/// allocation and one ingest descriptor (the reference's per-packet
/// siamese_encoder_add, siamese.cpp:96-108).
SIAMESE_EXPORT SiameseResult sgpu_encoder_add_range(SgpuEncoder encoder, const void* deviceData, size_t stride,
                                                    const unsigned* bytes, unsigned fixedBytes, unsigned count,
                                                    unsigned* firstPacketNumOut, unsigned* addedOut);
SIAMESE_EXPORT SiameseResult sgpu_encoder_remove_before(SgpuEncoder encoder, unsigned firstKept);
SIAMESE_EXPORT SiameseResult sgpu_encode(SgpuEncoder encoder, SgpuRecoveryPacket* out);
/// `count` sgpu_encode calls in one: out[k] = what the k-th call returns,
/// until a call does not succeed, whose result is returned (Success if none
/// failed; that call's out[k].DataBytes = 0); *producedOut = packets made.
/// Every packet of the call stays valid until the next sgpu_encode /
/// sgpu_encode_range on the same encoder.  Bit-exact with the single calls
/// (the reference's siamese_encode, siamese.cpp:159-168, per packet,
/// SiameseEncoder.cpp:1146-1254): a block-mode sender that knows how many
/// recovery packets it needs asks for them in one call.
SIAMESE_EXPORT SiameseResult sgpu_encode_range(SgpuEncoder encoder, SgpuRecoveryPacket* out, unsigned count,
                                               unsigned* producedOut);

SIAMESE_EXPORT SgpuDecoder sgpu_decoder_create(void);
SIAMESE_EXPORT void sgpu_decoder_free(SgpuDecoder decoder);
SIAMESE_EXPORT SiameseResult sgpu_decoder_add_original(SgpuDecoder decoder, unsigned packetNum,
                                                       const void* deviceData, unsigned bytes);
/// `count` sgpu_decoder_add_original calls in one: packet firstPacketNum + k
/// with its payload at deviceData + k * stride, bytes[k] bytes (fixedBytes
/// when bytes is NULL).  results[k] (optional) = call k's result; like the
/// calls, DuplicateData goes on and any other failure stops the run, its
/// result returned (Success if none stopped it); *callsOut = calls made.
/// (siamese_decoder_add_original, siamese.cpp:207-220, per packet.)
SIAMESE_EXPORT SiameseResult sgpu_decoder_add_original_range(SgpuDecoder decoder, unsigned firstPacketNum,
                                                             const void* deviceData, size_t stride,
                                                             const unsigned* bytes, unsigned fixedBytes,
                                                             unsigned count, SiameseResult* results,
                                                             unsigned* callsOut);
SIAMESE_EXPORT SiameseResult sgpu_decoder_add_recovery(SgpuDecoder decoder,
                                                       const SgpuRecoveryPacket* packet);
SIAMESE_EXPORT SiameseResult sgpu_decoder_is_ready(SgpuDecoder decoder);
SIAMESE_EXPORT SiameseResult sgpu_decode(SgpuDecoder decoder, SiameseOriginalPacket** packetsOut,
                                         unsigned* countOut);
/// sgpu_decode with the recovery matrix on the device: when the decode would
/// start a fresh elimination (GenerateMatrix + GaussianElimination,
/// reference SiameseDecoder.cpp:2157-2531) of at most 255 lost columns and
/// 256 recovery rows, the matrix job is queued and SGPU_DECODE_PENDING is
/// returned.  Flush (sgpu_flush, or wait for a later sgpu_enqueue ticket),
/// then call sgpu_decode_device again with the same arguments: it returns
/// what sgpu_decode would have returned, with the same outputs (an
/// elimination that stopped short of a pivot is repeated on the host, which
/// keeps the state the next attempt resumes from).  A square matrix of rows
/// of one length (a block decode) is chained: the elimination of received
/// data and the solve ride in the same submission, gated on the device
/// elimination's outcome, so the packets this second call returns already
/// carry their exact lengths.  While a job is pending, every other call on
/// this decoder returns Siamese_InvalidInput.  Any other decode runs as
/// sgpu_decode does.
#define SGPU_DECODE_PENDING ((SiameseResult)6)
SIAMESE_EXPORT SiameseResult sgpu_decode_device(SgpuDecoder decoder, SiameseOriginalPacket** packetsOut,
                                                unsigned* countOut);
/// Returns a device pointer; waits for outstanding work if the packet's
/// exact length is still being computed.
SIAMESE_EXPORT SiameseResult sgpu_decoder_get(SgpuDecoder decoder, SiameseOriginalPacket* packet);
/// sgpu_decoder_get for packets firstPacketNum, firstPacketNum + 1, ... into
/// packets[0, count) until one does not return Success; *gotOut = packets
/// returned.  Returns the result of the get that stopped (Success if none).
SIAMESE_EXPORT SiameseResult sgpu_decoder_get_range(SgpuDecoder decoder, unsigned firstPacketNum, unsigned count,
                                                    SiameseOriginalPacket* packets, unsigned* gotOut);
/// sgpu_decode without waiting (see "Deferred outputs" above): the recovered
/// packets are written to out[0, *countOut), PacketNum at once, Data and
/// DataBytes at once or when the solve's submission completes.  capacity must
/// be at least 255 (the most one solve recovers) and at least the packets
/// held by single-packet recoveries since the last decode; Siamese_InvalidInput
/// otherwise, with nothing consumed.
SIAMESE_EXPORT SiameseResult sgpu_decode_deferred(SgpuDecoder decoder, SiameseOriginalPacket* out,
                                                  unsigned capacity, unsigned* countOut);
/// sgpu_decoder_get without waiting: Success / NeedMoreData as
/// sgpu_decoder_get returns them; for a packet still being solved, *packet's
/// Data and DataBytes are written when the solve's submission completes.
SIAMESE_EXPORT SiameseResult sgpu_decoder_get_deferred(SgpuDecoder decoder, SiameseOriginalPacket* packet);
/// Non-blocking lookup: Success if the packet is present (length may still
/// be pending), NeedMoreData if not.
SIAMESE_EXPORT SiameseResult sgpu_decoder_has(SgpuDecoder decoder, unsigned packetNum);

/// Submit all queued device work of every instance and wait for it.
SIAMESE_EXPORT int sgpu_flush(void);
/// Submit, then complete the previous submission (one submission in flight).
SIAMESE_EXPORT int sgpu_submit(void);
/// Submit without waiting: returns the submission's ticket (>= 0; 0 when
/// nothing was ever queued), -1 once the device has failed.
SIAMESE_EXPORT long long sgpu_enqueue(void);
/// Wait for submission `ticket` and every earlier one; nonzero on a device
/// failure (sticky: every instance reports Siamese_Disabled afterwards).
SIAMESE_EXPORT int sgpu_wait(long long ticket);
/// Non-blocking: 1 if submission `ticket` has completed (as sgpu_wait would
/// return), 0 if it is still in flight, -1 once the device has failed.
SIAMESE_EXPORT int sgpu_query(long long ticket);
/// Run fn(ctx, i) for i in [0, count) on the library's host worker threads
/// (the caller takes part) and return when all calls are done.  Lets an
/// application drive many instances on the threads the library placed next
/// to the GPU.
SIAMESE_EXPORT void sgpu_parallel_for(unsigned count, void (*fn)(void* ctx, unsigned index),
                                      void* ctx);

/// Device memory helpers for applications and the benchmark harness.
SIAMESE_EXPORT void* sgpu_device_alloc(size_t bytes);
SIAMESE_EXPORT void sgpu_device_free(void* p);
/// Page-locked host memory (packet staging for DMA to and from the GPU).
SIAMESE_EXPORT void* sgpu_host_alloc(size_t bytes);
SIAMESE_EXPORT void sgpu_host_free(void* p);
SIAMESE_EXPORT int sgpu_h2d(void* deviceDst, const void* hostSrc, size_t bytes);
/// Gather `count` device ranges into one host buffer (concatenated in order).
/// Runs immediately; queued-but-unflushed codec work is left untouched.
SIAMESE_EXPORT int sgpu_gather(unsigned count, const void* const* deviceSrcs, const unsigned* bytes,
                               void* hostOut);

/// Asynchronous host -> device copy for packets arriving in pinned host
/// memory: issued at once on the library's staging stream; every submission
/// enqueued after this call waits for it on the device (the host never
/// blocks), so the copy overlaps the device work already in flight.  The
/// caller guarantees that no unfinished submission reads or writes deviceDst.
SIAMESE_EXPORT int sgpu_h2d_async(void* deviceDst, const void* hostSrc, size_t bytes);
/// Gather `count` device ranges produced by COMPLETED submissions into pinned
/// host memory (sgpu_host_alloc) on the library's gather stream, without
/// waiting for submissions still in flight.  Range i lands at offset
/// sum over k < i of align16(bytes[k]) (16-byte aligned, one DMA for all).
SIAMESE_EXPORT int sgpu_gather_completed(unsigned count, const void* const* deviceSrcs, const unsigned* bytes,
                                         void* pinnedOut);
/// sgpu_gather_completed without waiting for the copy: returns a gather
/// ticket (> 0; -1 on failure) at once.  The sources are read before the
/// device work of any later submission runs (that work waits for them on the
/// device), so the instances owning them may be driven on right away;
/// pinnedOut holds the bytes once sgpu_gather_wait(ticket) returns 0.  May
/// run beside instance calls, like sgpu_gather_completed.
SIAMESE_EXPORT long long sgpu_gather_async(unsigned count, const void* const* deviceSrcs, const unsigned* bytes,
                                           void* pinnedOut);
/// Wait until gather `ticket` and every earlier one have landed in host
/// memory.  0 on success, -1 after a device fault.
SIAMESE_EXPORT int sgpu_gather_wait(long long ticket);

/*
    Framed datagrams: packet ingest and egress in bulk (the UDP side of an
    application; replaces nothing in siamese.h).  A frame carries one
    datagram:
      [L: byte length of the rest, in the symbol length-prefix format of
          the reference (SiameseSerializers.h:566-593), 1-4 bytes]
      [type: 1 byte, SGPU_FRAME_ORIGINAL or SGPU_FRAME_RECOVERY]
      [flow: 3 bytes little-endian, the application's stream id]
      original:  [PacketNum: 3 bytes LE] [payload]
      recovery:  [the recovery packet, its metadata footer included
                  (SiameseSerializers.h:736-800)]
    Frames follow each other directly; a zero byte where a frame would start
    is an empty frame and is skipped (senders pad frames with zeros).
*/
#define SGPU_FRAME_ORIGINAL 0
#define SGPU_FRAME_RECOVERY 1

typedef struct SgpuFrame
{
    unsigned Type;        ///< SGPU_FRAME_ORIGINAL / SGPU_FRAME_RECOVERY
    unsigned Flow;
    unsigned PacketNum;   ///< originals
    unsigned Offset;      ///< byte offset of the data (payload / recovery packet) in the buffer
    unsigned Bytes;       ///< data bytes
} SgpuFrame;

/// Header bytes a frame of `type` carrying `dataBytes` puts before its data.
SIAMESE_EXPORT unsigned sgpu_frame_header_bytes(unsigned type, unsigned dataBytes);
/// Write a frame header to `out` (sgpu_frame_header_bytes bytes); the data
/// follows it.  Returns the header size, 0 on invalid input.
SIAMESE_EXPORT unsigned sgpu_frame_write_header(unsigned type, unsigned flow, unsigned packetNum,
                                                unsigned dataBytes, void* out);
/// Parse up to maxFrames frames of frames[0, bytes) (host memory, bytes <
/// 4 GiB).  InvalidInput on a malformed frame or when more frames remain;
/// the frames before a malformed one are still returned (*countOut).
SIAMESE_EXPORT SiameseResult sgpu_frames_parse(const void* frames, size_t bytes, SgpuFrame* out,
                                               unsigned maxFrames, unsigned* countOut);
/// Packet ingest: the frames in hostFrames[0, bytes) (pinned host memory)
/// whose identical copy the caller staged at deviceFrames with
/// sgpu_h2d_async.  Parses them in bulk and hands each datagram to
/// decoders[flow]: originals to sgpu_decoder_add_original, recovery packets
/// to sgpu_decoder_add_recovery (footer and head read from the host copy,
/// the bytes copied from the device copy by the next submission, which
/// waits for the staging copy on the device).  results[i] (optional) is the
/// call's result for frame i (InvalidInput for a flow without a decoder).
/// A malformed frame ends the call: every frame before it is delivered and
/// counted in *countOut, and the call returns InvalidInput.  bytes < 4 GiB.
/// The decoders must not be driven concurrently with this call; deviceFrames
/// stays untouched until the next submission has completed.
SIAMESE_EXPORT SiameseResult sgpu_frames_recv(const SgpuDecoder* decoders, unsigned decoderCount,
                                              const void* hostFrames, const void* deviceFrames, size_t bytes,
                                              SiameseResult* results, unsigned maxFrames, unsigned* countOut);
/// Packet egress: frame `count` recovery packets (flows[i] their stream ids)
/// into pinned host memory without waiting (a gather, as
/// sgpu_gather_async: same lifetime rule for the packets).  Frame i starts
/// at a 16-byte boundary, zero padding between frames.  *bytesOut = the
/// frame stream's length (<= capacity).  Returns a gather ticket for
/// sgpu_gather_wait, -1 on failure (capacity too small, a packet of 0 or more
/// than SIAMESE_MAX_PACKET_BYTES bytes, device fault).
SIAMESE_EXPORT long long sgpu_frames_send(unsigned count, const SgpuRecoveryPacket* packets, const unsigned* flows,
                                          void* pinnedOut, size_t capacity, size_t* bytesOut);

/// Device timing of flushed work since the last reset (milliseconds).
SIAMESE_EXPORT void sgpu_timing(int enable, int reset, double* execMs, double* totalMs);
/// Device milliseconds per kernel class since the last sgpu_timing reset,
/// while timing is enabled: [0] k_ingest, [1] k_exec, [2] k_ldpc, [3] the
/// solve kernels (k_solve_pre + k_solve_tr + k_solve_main on launches of
/// >= 16 solves, k_solve_main alone below that), [4] k_ge (sgpu_decode_device);
/// count entries at most.
SIAMESE_EXPORT void sgpu_timing_kernels(double* msOut, unsigned count);
/// Engine counters (15 values): flushes, launches, ops, terms, solves,
/// ingests, upload bytes, algorithmic op bytes, algorithmic output bytes,
/// the part of the algorithmic bytes handled by the solve kernels, then host
/// nanoseconds spent assembling flushes, waiting for the device,
/// running completions, and reclaiming released buffers, then the number of
/// executor launches.
SIAMESE_EXPORT void sgpu_engine_stats(uint64_t* out15);
/// sgpu_engine_stats' 15 values, then the algorithmic bytes of k_ldpc (the
/// wide rows' picks, part of the algorithmic op bytes), then the executor
/// launches' compulsory bytes (see sgpu_measure_unique), then the device
/// recovery-matrix jobs (sgpu_decode_device), those of them chained into
/// their decode's submission, and the chained ones whose matrix was singular
/// (the host repeated the elimination); count entries at most.
SIAMESE_EXPORT void sgpu_engine_stats_ex(uint64_t* out, unsigned count);
/// Measurement aid: while on, flush assembly counts the executor launches'
/// compulsory bytes -- each distinct source symbol read once, each
/// destination written once, the op stream once -- into sgpu_engine_stats_ex
/// [16].  The algorithmic bytes count every re-read of a symbol the reference
/// performs; this is the traffic a kernel that re-reads nothing from HBM
/// would move.  Off by default (it sorts every segment's operands).
SIAMESE_EXPORT void sgpu_measure_unique(int on);

/// Device bytes the engine's symbol arena has taken from hipMalloc so far
/// (grows while warming up, then stays flat: buffers are recycled).
SIAMESE_EXPORT uint64_t sgpu_arena_bytes(void);
/// Keep at least `bytes` of untouched arena memory in reserve (allocated now,
/// counted in sgpu_arena_bytes), so later growth of the working set takes it
/// instead of calling hipMalloc inside a latency-sensitive phase.
SIAMESE_EXPORT int sgpu_arena_reserve(size_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* SIAMESE_GPU_H */
