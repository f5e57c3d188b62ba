"""Randomised call-sequence comparison of two siamese.h implementations.

A seeded scenario drives one encoder/decoder pair of each library with the
same calls -- variable and tiny packet sizes, losses, reordering, duplicates
of originals and recovery packets, acknowledgements (decoder_ack ->
encoder_ack), remove_before, get -- and records every result code and every
returned byte string.  Two implementations agree iff the records are equal.
"""
import hashlib
import random

from siamese_amd.binding import Success


def _h(b):
    return None if b is None else (len(b), hashlib.blake2b(b, digest_size=8).hexdigest())


def run(lib, seed, steps=1500, max_bytes=1500):
    rnd = random.Random(seed)
    enc = lib.Encoder()
    dec = lib.Decoder()
    log = []
    held_orig = []      # originals delayed for out-of-order delivery
    held_rec = []       # recovery packets delayed
    sent = {}           # packet num -> data
    loss = rnd.choice([0.02, 0.1, 0.25])
    for step in range(steps):
        op = rnd.random()
        if op < 0.55:
            n = rnd.choice([1, 2, 3, 17, 100, 1400, rnd.randint(1, max_bytes),
                            rnd.randint(1, max_bytes), 3000 if rnd.random() < 0.02 else 64])
            data = bytes(rnd.getrandbits(8) for _ in range(n))
            rc, num = enc.add_raw(data)
            log.append(("add", rc, num))
            if rc != Success:
                continue
            sent[num] = data
            r = rnd.random()
            if r < loss:
                continue
            if r < loss + 0.05:
                held_orig.append((num, data))
                continue
            log.append(("add_orig", dec.add_original(num, data)))
            if rnd.random() < 0.03:
                log.append(("dup_orig", dec.add_original(num, data)))
        elif op < 0.80:
            rc, rec = enc.encode_raw()
            log.append(("encode", rc, _h(rec)))
            if rec is None:
                continue
            r = rnd.random()
            if r < loss:
                continue
            if r < loss + 0.05:
                held_rec.append(rec)
                continue
            log.append(("add_rec", dec.add_recovery(rec)))
            if rnd.random() < 0.03:
                log.append(("dup_rec", dec.add_recovery(rec)))
            for _ in range(4):
                ready = dec.is_ready()
                log.append(("ready", ready))
                if ready != Success:
                    break
                rc, pkts = dec.decode_raw()
                log.append(("decode", rc, None if pkts is None else [(p, _h(d)) for p, d in pkts]))
                if pkts:
                    for p, d in pkts:
                        assert d == sent.get(p), "recovered packet %d corrupt" % p
        elif op < 0.86 and held_orig:
            num, data = held_orig.pop(rnd.randrange(len(held_orig)))
            log.append(("late_orig", dec.add_original(num, data)))
        elif op < 0.90 and held_rec:
            rec = held_rec.pop(rnd.randrange(len(held_rec)))
            log.append(("late_rec", dec.add_recovery(rec)))
        elif op < 0.94:
            rc, msg = dec.ack()
            log.append(("dec_ack", rc, _h(msg)))
            if msg and rnd.random() < 0.8:
                log.append(("enc_ack",) + enc.ack(msg))
        elif op < 0.97:
            num = rnd.randrange(0, max(1, len(sent) + 8))
            rc1, d1 = enc.get(num)
            rc2, d2 = dec.get(num)
            log.append(("get", num, rc1, _h(d1), rc2, _h(d2)))
        else:
            if sent:
                num = rnd.randrange(0, len(sent) + 1)
                log.append(("remove_before", num, enc.remove_before(num)))
    log.append(("enc_stats", enc.stats()[:8]))
    log.append(("dec_stats", dec.stats()[:10]))
    enc.close()
    dec.close()
    return log


def run_arq(lib, seed, rounds=3, sleep_s=0.65):
    """ARQ scenario past the retransmission timeout (reference
    SiameseEncoder.cpp:835-1044, :514-800): originals over a lossy link, the
    decoder's NACK acknowledgement fed to the encoder, then after sleeping
    beyond any RTO (500 ms initial, 1.5 x max RTT >= 20 ms later) every
    retransmission the encoder offers, with its bytes, some of them
    delivered.  Retransmit is only called right after a sleep, so the
    sequence does not depend on how long the calls themselves take."""
    import time
    rnd = random.Random(seed)
    enc = lib.Encoder()
    dec = lib.Decoder()
    log = []
    sent = {}
    for _ in range(rounds):
        loss = rnd.choice([0.1, 0.2, 0.35])
        for _ in range(rnd.randint(20, 90)):
            n = rnd.choice([1, 40, 700, 1400, rnd.randint(1, 1500)])
            data = bytes(rnd.getrandbits(8) for _ in range(n))
            rc, num = enc.add_raw(data)
            log.append(("add", rc, num))
            if rc != Success:
                continue
            sent[num] = data
            if rnd.random() >= loss:
                log.append(("add_orig", dec.add_original(num, data)))
        if rnd.random() < 0.5:
            rc, rec = enc.encode_raw()
            log.append(("encode", rc, _h(rec)))
            if rec is not None:
                log.append(("add_rec", dec.add_recovery(rec)))
        rc, msg = dec.ack()
        log.append(("dec_ack", rc, _h(msg)))
        if msg:
            log.append(("enc_ack",) + enc.ack(msg))
        time.sleep(sleep_s)
        for _ in range(400):
            rc, r = enc.retransmit()
            log.append(("retransmit", rc, None if r is None else (r[0], _h(r[1]))))
            if rc != Success:
                break
            assert r[1] == sent.get(r[0]), "retransmitted packet %d corrupt" % r[0]
            if rnd.random() < 0.7:
                log.append(("add_orig", dec.add_original(r[0], r[1])))
        if rnd.random() < 0.3 and sent:
            num = rnd.randrange(0, len(sent))
            log.append(("remove_before", num, enc.remove_before(num)))
    log.append(("enc_stats", enc.stats()[:8]))
    log.append(("dec_stats", dec.stats()[:10]))
    enc.close()
    dec.close()
    return log


def normalise(log):
    import json
    return json.loads(json.dumps(log))


def run_isolated(library_path, seed, steps=1500, scenario="run"):
    """Run the scenario in a child process (the reference can crash on some
    sequences); returns the normalised log or None if the child died."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    args = "%d, %d" % (seed, steps) if scenario == "run" else "%d" % seed
    code = ("import sys, json; sys.path[:0] = [%r, %r]; import api_fuzz; "
            "from siamese_amd.binding import SiameseLib; "
            "print(json.dumps(api_fuzz.%s(SiameseLib(%r).init(), %s)))"
            % (here, os.path.dirname(here), scenario, library_path, args))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    if p.returncode != 0:
        return None
    return json.loads(p.stdout)


def first_difference(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x, y
    if len(a) != len(b):
        return min(len(a), len(b)), "len %d" % len(a), "len %d" % len(b)
    return None
