// frames.cpp -- see frames.h.
#include "frames.h"
#include "codedef.h"

namespace sgpu {

namespace {
constexpr unsigned kOriginalHeader = 1 + kFrameFlowBytes + 3;   // type, flow, PacketNum
constexpr unsigned kRecoveryHeader = 1 + kFrameFlowBytes;       // type, flow

inline unsigned prefix_bytes(unsigned length)
{
    return length < 0x80 ? 1 : length < 0x4000 ? 2 : length < 0x200000 ? 3 : 4;
}
} // namespace

unsigned frame_header_bytes(unsigned type, unsigned dataBytes)
{
    const unsigned inner = (type == kFrameOriginal ? kOriginalHeader : kRecoveryHeader);
    return prefix_bytes(inner + dataBytes) + inner;
}

unsigned frame_write_header(unsigned type, unsigned flow, unsigned packetNum, unsigned dataBytes, uint8_t* out)
{
    const unsigned inner = (type == kFrameOriginal ? kOriginalHeader : kRecoveryHeader);
    unsigned n = write_length_prefix(inner + dataBytes, out);
    out[n++] = (uint8_t)type;
    out[n++] = (uint8_t)flow;
    out[n++] = (uint8_t)(flow >> 8);
    out[n++] = (uint8_t)(flow >> 16);
    if (type == kFrameOriginal) {
        out[n++] = (uint8_t)packetNum;
        out[n++] = (uint8_t)(packetNum >> 8);
        out[n++] = (uint8_t)(packetNum >> 16);
    }
    return n;
}

long frames_parse(const uint8_t* buf, size_t bytes, FrameInfo* out, size_t maxFrames, size_t* consumed,
                  size_t* badOffset)
{
    size_t at = 0, n = 0;
    *badOffset = kNoBadFrame;
    while (at < bytes && n < maxFrames) {
        if (buf[at] == 0) {   // empty frame: padding
            ++at;
            continue;
        }
        const size_t left = bytes - at;
        unsigned length = 0;
        const int h = read_length_prefix(buf + at, left < 4 ? (unsigned)left : 4u, &length);
        if (h < 1 || (size_t)h + length > left || length < 1) {
            *badOffset = at;
            break;
        }
        const uint8_t* f = buf + at + h;
        FrameInfo& fi = out[n];
        fi.type = f[0];
        if (fi.type == kFrameOriginal) {
            if (length <= kOriginalHeader) {
                *badOffset = at;
                break;
            }
            fi.flow = f[1] | ((uint32_t)f[2] << 8) | ((uint32_t)f[3] << 16);
            fi.packetNum = f[4] | ((uint32_t)f[5] << 8) | ((uint32_t)f[6] << 16);
            fi.offset = (uint32_t)(at + h + kOriginalHeader);
            fi.bytes = length - kOriginalHeader;
        } else if (fi.type == kFrameRecovery) {
            if (length <= kRecoveryHeader) {
                *badOffset = at;
                break;
            }
            fi.flow = f[1] | ((uint32_t)f[2] << 8) | ((uint32_t)f[3] << 16);
            fi.packetNum = 0;
            fi.offset = (uint32_t)(at + h + kRecoveryHeader);
            fi.bytes = length - kRecoveryHeader;
        } else {
            *badOffset = at;
            break;
        }
        ++n;
        at += (size_t)h + length;
    }
    // trailing padding after the last frame counts as consumed
    while (at < bytes && n == maxFrames && buf[at] == 0)
        ++at;
    *consumed = at;
    return (long)n;
}

} // namespace sgpu
