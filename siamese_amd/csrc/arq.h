// arq.h -- the selective-acknowledgement (NACK) side channel: wire formats,
// the windowed-maximum RTT tracker and the encoder's acknowledgement state.
// Pure host logic with no symbol arithmetic (reference SiameseSerializers.h:
// 320-375 and 807-994, SiameseTools.h:134-236, SiameseEncoder.h:239-327).
#pragma once

#include <cstdint>
#include <vector>

namespace sgpu {

uint64_t now_msec();

constexpr unsigned kMaxNackRangeBytes = 7;

/// Packet number in front-of-buffer form, 1-3 bytes (SiameseSerializers.h:330-375).
inline unsigned put_packetnum_head(unsigned num, uint8_t* out)
{
    if (num < 0x80) {
        out[0] = (uint8_t)num;
        return 1;
    }
    if (num < 0x4000) {
        out[0] = (uint8_t)(0x80 | (num >> 8));
        out[1] = (uint8_t)num;
        return 2;
    }
    out[0] = (uint8_t)(0xC0 | (num >> 16));
    out[1] = (uint8_t)(num >> 8);
    out[2] = (uint8_t)num;
    return 3;
}

inline int get_packetnum_head(const uint8_t* in, int avail, unsigned* num)
{
    if (!in || avail < 1)
        return -1;
    const int width = in[0] >> 6;
    if (width <= 1) {
        *num = in[0];
        return 1;
    }
    if (avail < width)
        return -1;
    if (width == 2)
        *num = (((unsigned)in[0] << 8) | in[1]) & 0x3fff;
    else
        *num = (((unsigned)in[0] << 16) | ((unsigned)in[1] << 8) | in[2]) & 0x3fffff;
    return width;
}

/// One NACK loss range: CC X NNNNN + up to 3 extension bytes of the relative
/// start, then an optional 1-3 byte extended loss count (:854-930).
unsigned put_nack_range(unsigned relativeStart, unsigned lossCountM1, uint8_t* out);
int get_nack_range(const uint8_t* in, unsigned avail, unsigned* relativeStart, unsigned* lossCountM1);

/// Running windowed maximum over 3 samples (SiameseTools.h:134-236).
struct WindowedMax
{
    struct Sample
    {
        unsigned value = 0;
        uint64_t time = 0;
        bool expired(uint64_t now, uint64_t timeout) const { return now - time > timeout; }
    } s[3];
    unsigned best() const { return s[0].value; }
    void reset(Sample x) { s[0] = s[1] = s[2] = x; }
    void update(unsigned value, uint64_t now, uint64_t window);
};

/// Encoder-side view of the latest acknowledgement (SiameseEncoder.h:239-327).
struct AckState
{
    std::vector<uint8_t> data;     // NACK ranges + padding
    unsigned dataBytes = 0;
    static constexpr unsigned kPadding = 8;
    unsigned offset = 0;
    unsigned lossColumn = 0;
    unsigned lossCount = 0;
    unsigned nextColumnExpected = 0;
    unsigned nextRtoColumn = 0;
    bool foundOldest = false;
    unsigned oldestColumn = 0;
    unsigned rtoMsec = 500;
    WindowedMax maxRtt;

    bool decode_next_range();
    bool next_loss_column(unsigned* column);
    void restart_iterator();
};

} // namespace sgpu
