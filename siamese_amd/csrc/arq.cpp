// arq.cpp -- NACK side channel (see arq.h) plus the ARQ members of the
// encoder and decoder control planes.  Host-only; no device work.
#include "arq.h"

#include "codedef.h"
#include "decoder.h"
#include "encoder.h"

#include <ctime>
#include <cstring>

namespace sgpu {

uint64_t now_msec()
{
    // Every add stamps its original (reference SiameseEncoder.cpp:142); the
    // coarse monotonic clock is a memory read (no vDSO/TSC round trip) and
    // its tick is far below the millisecond-scale RTO arithmetic it feeds.
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
    return (uint64_t)ts.tv_sec * 1000u + (uint64_t)ts.tv_nsec / 1000000u;
}

unsigned put_nack_range(unsigned relativeStart, unsigned lossCountM1, uint8_t* out)
{
    unsigned b0 = (lossCountM1 <= 2 ? lossCountM1 : 3) | (relativeStart << 3);
    unsigned n = 1;
    if (relativeStart >= (1u << 5)) {
        unsigned b1 = relativeStart >> 5;
        if (relativeStart >= (1u << 12)) {
            unsigned b2 = relativeStart >> 12;
            if (relativeStart >= (1u << 19)) {
                out[3] = (uint8_t)(relativeStart >> 19);
                b2 |= 0x80;
                ++n;
            }
            out[2] = (uint8_t)b2;
            b1 |= 0x80;
            ++n;
        }
        out[1] = (uint8_t)b1;
        b0 |= 4;
        ++n;
    }
    out[0] = (uint8_t)b0;
    if (lossCountM1 >= 3) {
        uint8_t* ext = out + n;
        const unsigned extra = lossCountM1 - 3;
        unsigned e1 = extra;
        if (extra >= (1u << 7)) {
            unsigned e2 = extra >> 7;
            if (extra >= (1u << 14)) {
                ext[2] = (uint8_t)(extra >> 14);
                e2 |= 0x80;
                ++n;
            }
            ext[1] = (uint8_t)e2;
            e1 |= 0x80;
            ++n;
        }
        ext[0] = (uint8_t)e1;
        ++n;
    }
    return n;
}

int get_nack_range(const uint8_t* in, unsigned avail, unsigned* relativeStart, unsigned* lossCountM1)
{
    if (!in || avail < kMaxNackRangeBytes)
        return -1;
    const unsigned b0 = in[0];
    unsigned loss = b0 & 3;
    unsigned rel = b0 >> 3;
    unsigned n = 1;
    if (b0 & 4) {
        ++n;
        rel |= (in[1] & 0x7fu) << 5;
        if (in[1] & 0x80) {
            ++n;
            rel |= (in[2] & 0x7fu) << 12;
            if (in[2] & 0x80) {
                ++n;
                rel |= (unsigned)in[3] << 19;
            }
        }
    }
    if (loss == 3) {
        const uint8_t* ext = in + n;
        loss += ext[0] & 0x7f;
        if (ext[0] & 0x80) {
            loss += (ext[1] & 0x7fu) << 7;
            if (ext[1] & 0x80) {
                loss += (unsigned)ext[2] << 14;
                ++n;
            }
            ++n;
        }
        ++n;
    }
    *relativeStart = rel;
    *lossCountM1 = loss;
    return (int)n;
}

void WindowedMax::update(unsigned value, uint64_t now, uint64_t window)
{
    Sample x;
    x.value = value;
    x.time = now;
    if (s[0].value == 0 || value >= s[0].value || s[2].expired(now, window)) {
        reset(x);
        return;
    }
    if (value >= s[1].value)
        s[2] = s[1] = x;
    else if (value >= s[2].value)
        s[2] = x;
    if (s[0].expired(now, window)) {
        if (s[1].expired(now, window)) {
            s[0] = s[2];
            s[1] = x;
        } else {
            s[0] = s[1];
            s[1] = s[2];
        }
        s[2] = x;
        return;
    }
    if (s[1].value == s[0].value && s[1].expired(now, window / 4)) {
        s[2] = s[1] = x;
        return;
    }
    if (s[2].value == s[1].value && s[2].expired(now, window / 2))
        s[2] = x;
}

bool AckState::decode_next_range()
{
    if (offset >= dataBytes)
        return false;
    unsigned rel = 0, lossM1 = 0;
    const int w = get_nack_range(data.data() + offset, dataBytes + kPadding - offset, &rel, &lossM1);
    if (w < 0)
        return false;
    offset += w;
    if (offset > dataBytes)
        return false;
    lossColumn = column_add(lossColumn, rel);
    lossCount = lossM1 + 1;
    return true;
}

bool AckState::next_loss_column(unsigned* column)
{
    if (lossCount == 0) {
        lossColumn = column_add(lossColumn, 1);
        if (!decode_next_range())
            return false;
    }
    *column = lossColumn;
    lossColumn = column_add(lossColumn, 1);
    --lossCount;
    return true;
}

void AckState::restart_iterator()
{
    offset = 0;
    lossColumn = nextColumnExpected;
    lossCount = 0;
    decode_next_range();
}

// ---------------------------------------------------------------------------
// Encoder ARQ (reference SiameseEncoder.cpp:514-1044)

void EncoderCore::update_rto()
{
    const unsigned count = count_;
    unsigned firstLoss = column_to_element(ack_.nextColumnExpected);
    if (firstLoss >= count)
        return;
    const uint64_t now64 = now_msec();
    const uint32_t now = (uint32_t)now64;
    unsigned longest = 0;
    unsigned element = column_to_element(ack_.nextRtoColumn);
    if (element >= count)
        element = firstUnremoved_;

    auto sample = [&](unsigned e) {
        const int32_t delay = (int32_t)(now - slot(e).lastSend);
        if ((unsigned)delay > longest && delay > 0)
            longest = (unsigned)delay;
    };
    for (; element < firstLoss; ++element)
        sample(element);

    unsigned remaining = ack_.dataBytes;
    const uint8_t* p = ack_.data.data();
    while (remaining > 0) {
        unsigned rel = 0, lossM1 = 0;
        const int w = get_nack_range(p, remaining + AckState::kPadding, &rel, &lossM1);
        if (w < 0 || w > (int)remaining)
            return;
        p += w;
        remaining -= w;
        if (element + 1 < firstLoss)
            element = firstLoss - 1;
        firstLoss += rel;
        for (; element < firstLoss; ++element) {
            if (element >= count)
                return;
            sample(element);
        }
        firstLoss += lossM1 + 2;
    }
    ack_.nextRtoColumn = element_to_column(element);
    if (longest == 0)
        return;
    uint64_t window = (uint64_t)ack_.rtoMsec * 2;
    if (window < 100)
        window = 100;
    else if (window > 4000)
        window = 4000;
    ack_.maxRtt.update(longest, now64, window);
    ack_.rtoMsec = (ack_.maxRtt.best() * 3) / 2;
    if (ack_.rtoMsec < 20)
        ack_.rtoMsec = 20;
}

SiameseResult EncoderCore::acknowledge(const uint8_t* data, unsigned bytes, unsigned& nextExpectedOut)
{
    if (dead())
        return Siamese_Disabled;
    unsigned next = 0;
    const int h = get_packetnum_head(data, (int)bytes, &next);
    if (h < 1)
        return Siamese_InvalidInput;
    data += h;
    bytes -= h;

    bool process = true;
    if (column_delta_negative(column_sub(next, ack_.nextColumnExpected)))
        process = false; // stale acknowledgement
    else if (ack_.nextColumnExpected == next && !ack_.data.empty() && bytes == ack_.dataBytes &&
             std::memcmp(data, ack_.data.data(), bytes) == 0)
        process = false; // duplicate

    if (process) {
        ack_.nextColumnExpected = next;
        ack_.offset = 0;
        ack_.lossColumn = next;
        ack_.lossCount = 0;
        ack_.dataBytes = bytes;
        if (bytes > 0) {
            ack_.data.assign(data, data + bytes);
            ack_.data.resize(bytes + AckState::kPadding, 0);
            if (!ack_.decode_next_range())
                return Siamese_InvalidInput;
        }
        update_rto();
        remove_before(ack_.nextColumnExpected);
    }
    nextExpectedOut = ack_.nextColumnExpected;
    stats_[SiameseEncoderStats_AckCount]++;
    stats_[SiameseEncoderStats_AckBytes] += bytes + h;
    return Siamese_Success;
}

SiameseResult EncoderCore::retransmit_slot(EncSlot& s, SiameseOriginalPacket& out)
{
    out.PacketNum = s.column;
    out.Data = mirror_ ? s.host().data() + s.header : s.buf.ptr + s.header;
    out.DataBytes = s.bytes - s.header;
    if (out.DataBytes == 0) {
        disabled_ = true;
        return Siamese_Disabled;
    }
    stats_[SiameseEncoderStats_RetransmitCount]++;
    stats_[SiameseEncoderStats_RetransmitBytes] += out.DataBytes;
    return Siamese_Success;
}

SiameseResult EncoderCore::retransmit(SiameseOriginalPacket& out)
{
    out.Data = nullptr;
    out.DataBytes = 0;
    if (dead())
        return Siamese_Disabled;
    if (unacked() == 0) {
        ack_.foundOldest = false;
        return Siamese_NeedMoreData;
    }
    const unsigned first = column_sub(ack_.nextColumnExpected, columnStart_);
    const unsigned count = count_;
    if (column_delta_negative(first) || first < firstUnremoved_ || first >= count)
        return Siamese_NeedMoreData;

    const uint32_t now = (uint32_t)now_msec();
    const uint32_t rto = ack_.rtoMsec;

    if (ack_.foundOldest) {
        const unsigned e = column_sub(ack_.oldestColumn, columnStart_);
        if (!column_delta_negative(e) && e >= first && e < count) {
            EncSlot& s = slot(e);
            if ((uint32_t)(now - s.lastSend) < rto)
                return Siamese_NeedMoreData;
            s.lastSend = now;
            ack_.foundOldest = false;
            return retransmit_slot(s, out);
        }
        ack_.foundOldest = false;
    }

    unsigned nack = first;
    EncSlot* oldest = &slot(nack);
    uint32_t oldestSend = oldest->lastSend;
    if ((uint32_t)(now - oldestSend) >= rto) {
        oldest->lastSend = now;
        return retransmit_slot(*oldest, out);
    }

    if (ack_.dataBytes > 0) {
        ack_.restart_iterator();
        unsigned column = 0;
        while (ack_.next_loss_column(&column)) {
            nack = column_to_element(column);
            if (nack >= count)
                break;
            EncSlot& s = slot(nack);
            if ((uint32_t)(now - s.lastSend) >= rto) {
                s.lastSend = now;
                return retransmit_slot(s, out);
            }
            if ((int32_t)(oldestSend - s.lastSend) > 0) {
                oldest = &s;
                oldestSend = s.lastSend;
            }
        }
    }
    for (unsigned e = nack + 1; e < count; ++e) {
        EncSlot& s = slot(e);
        if ((uint32_t)(now - s.lastSend) >= rto) {
            s.lastSend = now;
            return retransmit_slot(s, out);
        }
        if ((int32_t)(oldestSend - s.lastSend) > 0) {
            oldest = &s;
            oldestSend = s.lastSend;
        }
    }
    ack_.foundOldest = true;
    ack_.oldestColumn = oldest->column;
    return Siamese_NeedMoreData;
}

// ---------------------------------------------------------------------------
// Decoder acknowledgement (reference SiameseDecoder.cpp:125-255)

unsigned DecoderCore::find_next_got(unsigned start)
{
    if (start >= count_)
        return count_;
    const unsigned subEnd = (count_ + kSubwindow - 1) / kSubwindow;
    unsigned sub = start / kSubwindow;
    unsigned bit = start % kSubwindow;
    while (sub < subEnd) {
        const DecSubwindow* sw = subwindows_[sub].get();
        if (sw->gotCount > 0) {
            const uint64_t bits = sw->got & (bit >= 64 ? 0 : (~0ULL << bit));
            if (bits) {
                const unsigned e = sub * kSubwindow + (unsigned)__builtin_ctzll(bits);
                return e > count_ ? count_ : e;
            }
        }
        bit = 0;
        ++sub;
    }
    return count_;
}

SiameseResult DecoderCore::acknowledgement(uint8_t* buffer, unsigned byteLimit, unsigned& usedBytes)
{
    settle();
    if (dead())
        return Siamese_Disabled;
    const unsigned count = count_;
    if (count == 0) {
        usedBytes = 0;
        return Siamese_NeedMoreData;
    }
    uint8_t* p = buffer;
    const unsigned nextElement = nextExpected_;
    const unsigned h = put_packetnum_head(element_to_column(nextElement), p);
    p += h;
    byteLimit -= h;
    if (nextElement < count) {
        unsigned offset = nextElement;
        while (byteLimit >= kMaxNackRangeBytes) {
            const unsigned start = find_next_lost(offset);
            if (start >= count) {
                if (count >= offset)
                    p += put_nack_range(count - offset, 0, p);
                break;
            }
            const unsigned end = find_next_got(start + 1);
            const unsigned w = put_nack_range(start - offset, end - start - 1, p);
            offset = end + 1;
            p += w;
            byteLimit -= w;
        }
    }
    usedBytes = (unsigned)(p - buffer);
    stats_[SiameseDecoderStats_AckCount]++;
    stats_[SiameseDecoderStats_AckBytes] += usedBytes;
    return Siamese_Success;
}

} // namespace sgpu
