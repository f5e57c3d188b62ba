// harness/scenario.h -- loopback workload definitions shared by every driver.
//
// This is the MI355X build's analogue of the reference's loopback simulator
// (reference tests/unit_test.cpp:79-125 payloads, :380-655 StreamingTest,
// :173-377 BlockRecoveryTest).  One "stream" is an encoder -> lossy channel ->
// decoder pipeline driven through the siamese.h call sequence.  The workload
// is a deterministic function of (config, global stream index), so the same
// stream run through the upstream reference (oracle/_ref), through the
// drop-in per-call API of libsiamese_amd, or through its batched device API
// must produce the same event digest -- that digest is the parity check.
//
// The per-stream logic is a resumable state machine (Stream::step) so the
// batched driver can advance thousands of streams in lock-step rounds while
// issuing exactly the same per-stream call sequence as the sequential driver.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace scen {

// PCG-XSH-RR 64/32, seeded the way the reference seeds it
// (reference SiameseTools.h:80-102).  Used for payloads and the loss channel.
struct Pcg
{
    uint64_t state = 0, inc = 0;
    void seed(uint64_t y, uint64_t x = 0)
    {
        state = 0;
        inc = (y << 1u) | 1u;
        next();
        state += x;
        next();
    }
    uint32_t next()
    {
        const uint64_t s = state;
        state = s * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((s >> 18) ^ s) >> 27);
        const uint32_t r = (uint32_t)(s >> 59);
        return (xs >> r) | (xs << ((32u - r) & 31u));
    }
};

// Variable packet size 2..1199 (reference unit_test.cpp:79-88)
inline unsigned variable_bytes(unsigned id)
{
    Pcg p;
    p.seed(id, 24124);
    return 2 + (p.next() % (1200 - 2));
}

// Self-validating payload: LE32 length then PCG(id, bytes) words
// (reference unit_test.cpp:90-116).
inline void fill_payload(unsigned id, uint8_t* buf, unsigned bytes)
{
    Pcg p;
    p.seed(id, bytes);
    if (bytes >= 4) {
        const uint32_t b = bytes;
        std::memcpy(buf, &b, 4);
        buf += 4;
        bytes -= 4;
    }
    while (bytes >= 4) {
        const uint32_t w = p.next();
        std::memcpy(buf, &w, 4);
        buf += 4;
        bytes -= 4;
    }
    if (bytes > 0) {
        uint32_t w = p.next();
        for (unsigned i = 0; i < bytes; ++i, w >>= 8)
            buf[i] = (uint8_t)w;
    }
}

struct Fnv
{
    uint64_t h = 1469598103934665603ULL;
    void bytes(const void* p, size_t n)
    {
        const uint8_t* b = (const uint8_t*)p;
        for (size_t i = 0; i < n; ++i) {
            h ^= b[i];
            h *= 1099511628211ULL;
        }
    }
    void u64(uint64_t v) { bytes(&v, 8); }
};

inline uint64_t hash_bytes(const void* p, size_t n)
{
    Fnv f;
    f.bytes(p, n);
    return f.h;
}

} // namespace scen

extern "C" {

/// Scenario knobs (ctypes-visible; keep POD, all uint32).
struct ScenarioConfig
{
    uint32_t block_mode;        ///< 0 = streaming, 1 = block (add all, then encode)
    uint32_t streams;           ///< streams simulated by this call
    uint32_t first_stream;      ///< global index of the first stream (sharding)
    uint32_t originals;         ///< originals per stream (N)
    uint32_t payload_bytes;     ///< fixed payload size; 0 = variable 2..1199
    uint32_t loss_pct;          ///< original loss percentage
    uint32_t recovery_loss_pct; ///< recovery loss percentage
    uint32_t recovery_interval; ///< streaming: encode when i % interval == phase
    uint32_t recovery_phase;
    uint32_t ack_policy;        ///< 0 none, 1 immediate remove_before, 2 lag-based
    uint32_t ack_lag;           ///< lag for policy 2
    uint32_t tail_limit;        ///< extra encodes after the last original / block limit
    uint32_t seed;              ///< loss channel seed (1013 = reference kSeed)
    uint32_t hash_data;         ///< 1: digests cover packet bytes; 0: lengths only
    uint32_t add_ranges;        ///< originals added by range calls (see Stream::add_ranges): block mode all
                                ///< at once; interleaved mode those up to each encode point
};

/// Per-stream outcome (ctypes-visible).
struct StreamResult
{
    uint64_t digest;            ///< FNV-1a-64 over the stream's event log
    uint64_t recovery_bytes;    ///< bytes of recovery packets emitted
    uint64_t payload_bytes;     ///< payload bytes of originals added
    uint32_t encodes;           ///< successful siamese_encode calls
    uint32_t recovery_lost;     ///< recovery packets dropped by the channel
    uint32_t originals_lost;    ///< originals dropped by the channel
    uint32_t recovered;         ///< packets returned by siamese_decode
    uint32_t decode_calls;
    uint32_t decode_fail;       ///< decode returned NeedMoreData
    uint32_t delivered;         ///< in-order deliveries (== originals when done)
    uint32_t status;            ///< 0 complete, 1 stalled, 2 api error, 3 data mismatch
};

} // extern "C"

namespace scen {

enum Event : uint64_t
{
    EV_ENC_ADD = 1, EV_DEC_ADD_ORIG, EV_ENCODE, EV_DEC_ADD_REC,
    EV_IS_READY, EV_DECODE, EV_DECODED_PKT, EV_GET, EV_REMOVE
};

inline uint64_t ev(uint64_t type, uint64_t result, uint64_t a = 0, uint64_t b = 0)
{
    return (type << 56) ^ (result << 48) ^ (a << 24) ^ b;
}

/*
    Codec concept (duck-typed) used by Stream<Codec>:

      bool needs_host_payload();              // false: payload already on device
      int  enc_add(unsigned id, const uint8_t* host, unsigned bytes, unsigned* packetNum);
      int  encode(Rec* rec);                  // Rec: driver-defined handle w/ .bytes
      int  dec_add_original(unsigned id, unsigned num, const uint8_t* host, unsigned bytes);
      int  dec_add_recovery(const Rec& rec);
      int  is_ready();
      int  decode(std::vector<Pkt>* out);     // Pkt: driver-defined w/ .num
      int  dec_get(unsigned num, Pkt* out);
      int  enc_remove_before(unsigned num);
      // Digest tokens: hash of (length || bytes) when cfg->hash_data, else the
      // length.  pkt_token also checks the bytes against the payload `id`.
      uint64_t rec_token(const Rec& rec);
      uint64_t pkt_token(const Pkt& p, unsigned id, bool* ok);
      bool wants_yield_after_decode();        // batch: lengths known after a flush
      bool outputs_final(const std::vector<Pkt>&);   // every decoded packet's length known

    Range calls (cfg->add_ranges; every codec supports them, a per-call API
    as loops of its single calls):

      int  enc_add_range(unsigned firstId, unsigned count, unsigned* firstNum, unsigned* added);
      int  dec_add_range(unsigned firstId, unsigned firstNum, unsigned count, int* results, unsigned* calls);
      int  dec_get_range(unsigned firstNum, unsigned count, Pkt* out, unsigned* got);
      void encode_hint(unsigned n);           // the next n encode() calls are sure to come
                                              // (a codec may make them in one range call)
*/

inline uint64_t data_token(bool hashData, const uint8_t* p, unsigned bytes)
{
    if (!hashData)
        return bytes;
    Fnv f;
    f.u64(bytes);
    f.bytes(p, bytes);
    return f.h;
}

template <class Codec, class Rec, class Pkt>
struct Stream
{
    enum Phase { ADD, ENCODE, DECODE_LOOP, DECODE_PENDING, DECODED, ACK, TAIL, DONE };
    /// codec decode(): a device matrix job was queued, call again after a flush
    static constexpr int kDecodePending = 6;

    const ScenarioConfig* cfg = nullptr;
    Codec* codec = nullptr;
    StreamResult* res = nullptr;
    unsigned global = 0;          // global stream index
    std::vector<uint64_t> log;    // event log
    bool logOn = true;            // keep the log (digests); off in timed bench steps
    void note(uint64_t e)
    {
        if (logOn)
            log.push_back(e);
    }

    Pcg loss;
    Phase phase = ADD;
    unsigned i = 0;               // next original index
    unsigned tail = 0;            // encodes issued after the originals
    unsigned encodedAhead = 0;    // block mode, ranges: tail count the last encode_hint covers
    unsigned nextExpected = 0;
    unsigned lastNum = 0;         // PacketNum of the most recent add
    unsigned recReceived = 0;     // recovery packets the decoder took
    bool tailMode = false;        // all originals added; only encodes remain
    std::vector<uint8_t> buf;
    std::vector<Pkt> decoded;     // output of the last successful decode
    std::vector<Pkt> getBuf;      // deliver_range's packets
    std::vector<uint8_t> lostBuf;  // add_ranges' loss draws (capacity reused)
    std::vector<int> resultsBuf;   // add_ranges' per-call results (capacity reused)
    bool dataOk = true;           // every returned packet matched its payload

    void init(const ScenarioConfig* c, Codec* k, StreamResult* r, unsigned globalIndex)
    {
        // (a recycled stream starts over: every field back to its initial
        // value, the vectors keeping their capacity)
        phase = ADD;
        i = tail = nextExpected = lastNum = recReceived = encodedAhead = 0;
        tailMode = false;
        dataOk = true;
        log.clear();
        decoded.clear();
        getBuf.clear();
        cfg = c;
        codec = k;
        res = r;
        global = globalIndex;
        std::memset(res, 0, sizeof(*res));
        if (logOn)
            log.reserve(4 * cfg->originals + 64);
        loss.seed(cfg->seed, global);
        buf.resize(cfg->payload_bytes ? cfg->payload_bytes + 8 : 1208);
        phase = ADD;
    }

    unsigned packet_id(unsigned index) const { return global * cfg->originals + index; }
    unsigned packet_bytes(unsigned id) const
    {
        return cfg->payload_bytes ? cfg->payload_bytes : variable_bytes(id);
    }

    bool done() const { return phase == DONE; }

    void fail(unsigned status)
    {
        res->status = status;
        phase = DONE;
    }

    // Pull every in-order packet already present at the decoder.
    bool deliver()
    {
        if (cfg->add_ranges)   // (one get_range: the same calls' results, the same log)
            return deliver_range();
        while (nextExpected < cfg->originals) {
            Pkt p;
            const int r = codec->dec_get(nextExpected, &p);
            if (r != 0) {
                note(ev(EV_GET, r, nextExpected));
                return r == 2; // NeedMoreData is the normal stop
            }
            note(ev(EV_GET, 0, nextExpected));
            note(codec->pkt_token(p, packet_id(nextExpected), &dataOk));
            ++nextExpected;
            ++res->delivered;
        }
        return true;
    }

    // Range form of deliver(): one get_range from nextExpected.
    bool deliver_range()
    {
        if (nextExpected >= cfg->originals)
            return true;
        std::vector<Pkt>& got = getBuf;
        got.resize(cfg->originals - nextExpected);
        unsigned n = 0;
        const int r = codec->dec_get_range(nextExpected, (unsigned)got.size(), got.data(), &n);
        for (unsigned k = 0; k < n; ++k) {
            note(ev(EV_GET, 0, nextExpected));
            note(codec->pkt_token(got[k], packet_id(nextExpected), &dataOk));
            ++nextExpected;
            ++res->delivered;
        }
        got.clear();
        if (r != 0)
            note(ev(EV_GET, r, nextExpected));
        return r == 0 || r == 2;
    }

    // Block mode, cfg->add_ranges: every original in range calls.  The
    // encoder takes them all in one call; the loss channel draws as the
    // per-call sequence does (one draw per original added, in order); each
    // run of consecutive received originals goes to the decoder in one call,
    // after which the in-order packets are delivered by one get_range.  The
    // event log records every call's observed results: the same events as
    // the per-call sequence, without its NeedMoreData probes of packets not
    // yet added (a run's deliveries are fetched once the run is in).
    void add_ranges(unsigned n)
    {
        unsigned first = 0, added = 0;
        const int r = codec->enc_add_range(packet_id(i), n, &first, &added);
        const unsigned i0 = i;
        std::vector<uint8_t>& lost = lostBuf;
        lost.assign(added, 0);
        for (unsigned k = 0; k < added; ++k) {
            const unsigned num = (first + k) & 0x3fffff;
            note(ev(EV_ENC_ADD, 0, num));
            res->payload_bytes += packet_bytes(packet_id(i0 + k));
            lost[k] = (loss.next() % 100) < cfg->loss_pct;
            if (lost[k])
                ++res->originals_lost;
        }
        lastNum = added ? ((first + added - 1) & 0x3fffff) : lastNum;
        if (r != 0) {
            note(ev(EV_ENC_ADD, r, 0));
            fail(2);
            return;
        }
        std::vector<int>& results = resultsBuf;
        for (unsigned k = 0; k < added;) {
            if (lost[k]) {
                ++k;
                continue;
            }
            unsigned e = k;
            while (e < added && !lost[e])
                ++e;
            const unsigned num0 = (first + k) & 0x3fffff;
            results.assign(e - k, 0);
            unsigned calls = 0;
            const int a = codec->dec_add_range(packet_id(i0 + k), num0, e - k, results.data(), &calls);
            for (unsigned j = 0; j < calls; ++j)
                note(ev(EV_DEC_ADD_ORIG, results[j], (num0 + j) & 0x3fffff));
            if ((a != 0 && a != 4) || calls != e - k) {
                fail(2);
                return;
            }
            if (nextExpected >= i0 + k && nextExpected < i0 + e && !deliver_range()) {
                fail(2);
                return;
            }
            k = e;
        }
        i += added;
    }

    // One encode + channel + add_recovery.
    void encode_once()
    {
        Rec rec;
        const int r = codec->encode(&rec);
        note(ev(EV_ENCODE, r));
        if (r == 2)
            return; // nothing to encode yet
        if (r != 0) {
            fail(2);
            return;
        }
        note(codec->rec_token(rec));
        ++res->encodes;
        res->recovery_bytes += rec.bytes;
        const bool lost = (loss.next() % 100) < cfg->recovery_loss_pct;
        if (lost) {
            ++res->recovery_lost;
            return;
        }
        const int a = codec->dec_add_recovery(rec);
        note(ev(EV_DEC_ADD_REC, a));
        if (a != 0) {
            fail(2);
            return;
        }
        ++recReceived;
        phase = DECODE_LOOP;
    }

    // The decode's outcome (one EV_DECODE per decode, however many calls it
    // took); the step's return value.
    bool decoded_result(int r)
    {
        note(ev(EV_DECODE, r, (uint64_t)decoded.size()));
        if (r == 2) {
            ++res->decode_fail;
            phase = DECODE_LOOP;
            return false;
        }
        if (r != 0) {
            fail(2);
            return false;
        }
        phase = DECODED;
        return codec->wants_yield_after_decode();
    }

    // Advance by one unit of work.  Returns true if the driver should stop
    // stepping this stream until outstanding device work has been flushed.
    bool step()
    {
        switch (phase) {
        case ADD: {
            if (i >= cfg->originals) {
                tailMode = true;
                phase = TAIL;
                return false;
            }
            if (cfg->add_ranges && cfg->block_mode) {
                add_ranges(cfg->originals - i);
                return false;
            }
            if (cfg->add_ranges) {
                // interleaved: the originals up to the next encode point in
                // one range call, then that encode, then one acknowledgement
                // (the per-call sequence acknowledges after every add)
                const unsigned iv = cfg->recovery_interval, ph = cfg->recovery_phase % iv;
                const unsigned toEncode = (ph + iv - i % iv) % iv;   // originals after i before the encode point
                const unsigned n = std::min(cfg->originals - i, toEncode + 1);
                add_ranges(n);
                if (res->status)
                    return false;
                phase = ((i - 1) % iv == ph) ? ENCODE : ACK;
                return false;
            }
            const unsigned id = packet_id(i);
            const unsigned bytes = packet_bytes(id);
            const uint8_t* host = nullptr;
            if (codec->needs_host_payload()) {
                fill_payload(id, buf.data(), bytes);
                host = buf.data();
            }
            unsigned num = 0;
            const int r = codec->enc_add(id, host, bytes, &num);
            note(ev(EV_ENC_ADD, r, num));
            if (r != 0) {
                fail(2);
                return false;
            }
            lastNum = num;
            res->payload_bytes += bytes;
            const bool lost = (loss.next() % 100) < cfg->loss_pct;
            if (lost) {
                ++res->originals_lost;
            } else {
                const int a = codec->dec_add_original(id, num, host, bytes);
                note(ev(EV_DEC_ADD_ORIG, a, num));
                if (a != 0 && a != 4) {
                    fail(2);
                    return false;
                }
                if (num == nextExpected && !deliver()) {
                    fail(2);
                    return false;
                }
            }
            ++i;
            if (cfg->block_mode) {
                phase = ADD;
                return false;
            }
            phase = ((i - 1) % cfg->recovery_interval == cfg->recovery_phase) ? ENCODE : ACK;
            return false;
        }
        case ENCODE:
            phase = ACK;
            encode_once();
            return codec->wants_yield_after_encode();
        case DECODE_LOOP: {
            const int ready = codec->is_ready();
            note(ev(EV_IS_READY, ready));
            if (ready != 0) {
                phase = tailMode ? TAIL : ACK;
                return false;
            }
            decoded.clear();
            ++res->decode_calls;
            const int r = codec->decode(&decoded);
            if (r == kDecodePending) {
                phase = DECODE_PENDING;
                return true;   // (its outcome arrives with the flush)
            }
            return decoded_result(r);
        }
        case DECODE_PENDING: {
            const int r = codec->decode(&decoded);
            if (r == kDecodePending)
                return true;
            // (a decode finished after its flush -- a chained device decode --
            // returns its packets with their lengths: no flush to wait for)
            const bool yield = decoded_result(r);
            return yield && !codec->outputs_final(decoded);
        }
        case DECODED: {
            for (const Pkt& p : decoded) {
                note(ev(EV_DECODED_PKT, 0, p.num));
                note(codec->pkt_token(p, packet_id(p.num), &dataOk));
                ++res->recovered;
            }
            decoded.clear();
            phase = DECODE_LOOP;
            if (!deliver())
                fail(2);
            return false;
        }
        case ACK: {
            phase = (i >= cfg->originals) ? TAIL : ADD;
            tailMode = (phase == TAIL);
            if (cfg->ack_policy == 1) {
                const int r = codec->enc_remove_before(nextExpected);
                note(ev(EV_REMOVE, r, nextExpected));
            } else if (cfg->ack_policy == 2) {
                const unsigned lag = (lastNum - nextExpected) & 0x3fffff;
                if (lag >= cfg->ack_lag && lag < 0x200000) {
                    const int r = codec->enc_remove_before(nextExpected);
                    note(ev(EV_REMOVE, r, nextExpected));
                }
            }
            return false;
        }
        case TAIL:
            if (nextExpected >= cfg->originals) {
                phase = DONE;
                return false;
            }
            if (tail >= cfg->tail_limit) {
                fail(1);
                return false;
            }
            if (cfg->add_ranges && cfg->block_mode && tail == encodedAhead) {
                // Block mode: the decoder cannot be ready before it holds as
                // many recovery packets as originals were lost (every row
                // covers the whole block, SiameseDecoder.cpp:541-600), so at
                // least that many more encodes follow, one per TAIL step,
                // whatever the channel drops; the codec may make them in one
                // range call.  The calls and their results are the per-call
                // sequence's (the encoder's state depends on its own calls
                // only), so the event log is unchanged.
                const unsigned lost = res->originals_lost;
                unsigned n = lost > recReceived ? lost - recReceived : 1;
                n = std::min(n, cfg->tail_limit - tail);
                encodedAhead = tail + n;
                codec->encode_hint(n);
            }
            ++tail;
            encode_once();
            return codec->wants_yield_after_encode();
        case DONE:
            return false;
        }
        return false;
    }

    void finish()
    {
        if (!dataOk && res->status == 0)
            res->status = 3;
        if (!logOn)
            return;   // no digest without a log
        Fnv f;
        for (uint64_t e : log)
            f.u64(e);
        f.u64(res->status);
        res->digest = f.h;
    }
};

} // namespace scen
