// frames.h -- framed datagrams: the wire format the batch API's packet
// ingest and egress use (include/siamese_gpu.h, "Framed datagrams").
//
// A frame carries one datagram:
//   [L: length of the rest, the symbol length prefix format
//       (reference SiameseSerializers.h:566-593), 1-4 bytes]
//   [type: 1 byte]  kFrameOriginal / kFrameRecovery
//   [flow: 3 bytes little-endian]  the application's stream id
//   original:  [PacketNum: 3 bytes LE (22 bits)] [payload]
//   recovery:  [the recovery packet: payload + its metadata footer
//               (reference SiameseSerializers.h:736-800)]
// Frames follow each other directly; a zero byte where a frame would start
// is an empty frame (L = 0) and is skipped, so senders may pad frames to
// any alignment with zeros (the egress gather places each frame at a 16-byte
// boundary).
#pragma once

#include <cstddef>
#include <cstdint>

namespace sgpu {

constexpr uint8_t kFrameOriginal = 0;
constexpr uint8_t kFrameRecovery = 1;
constexpr unsigned kFrameFlowBytes = 3;
constexpr unsigned kFrameMaxFlow = (1u << 24) - 1;

/// One parsed frame: byte offsets into the buffer it was parsed from.
struct FrameInfo
{
    uint32_t type;
    uint32_t flow;
    uint32_t packetNum;   // originals
    uint32_t offset;      // first data byte (payload, or the recovery packet)
    uint32_t bytes;       // data bytes
};

/// Header bytes before the data of a frame of `type` holding `dataBytes`.
unsigned frame_header_bytes(unsigned type, unsigned dataBytes);
/// Writes the header; returns its size (frame_header_bytes).
unsigned frame_write_header(unsigned type, unsigned flow, unsigned packetNum, unsigned dataBytes, uint8_t* out);
/// No malformed frame was met (frames_parse's *badOffset).
constexpr size_t kNoBadFrame = ~(size_t)0;
/// Parses frames from buf[0, bytes) (bytes < 4 GiB: offsets are 32-bit).
/// Returns the number of frames written to out (at most maxFrames).  Stops
/// at a malformed frame with *badOffset = where it starts (kNoBadFrame
/// otherwise): the frames before it are in out and *consumed = *badOffset.
/// Stops early (returning maxFrames) when out is full: *consumed says how far.
long frames_parse(const uint8_t* buf, size_t bytes, FrameInfo* out, size_t maxFrames, size_t* consumed,
                  size_t* badOffset);

} // namespace sgpu
