"""Golden fixtures: per-stream event digests of the upstream reference.

Each fixture under tests/golden/<name>.json holds the scenario config and the
digest of every stream as produced by oracle/_ref/libsiamese_ref.so (the
unmodified reference compiled from /root/reference) through the loopback
harness.  They are data (inputs + expected outputs); the generating script is
tests/golden/make_golden.py.  The GPU box has no /root/reference, so the GPU
tests compare against these when oracle/_ref is not shipped.
"""
import json
import os

import scenario_lib as S

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# name -> (base config, overrides).  hash_data=1 digests cover every byte of
# every recovery packet and recovered original; hash_data=0 digests cover the
# full call sequence, result codes and lengths (bytes are then checked against
# the self-validating payloads instead).
FIXTURES = {
    "smoke_C4x8": ("C4", dict(streams=8)),
    "C1": ("C1", dict()),
    "C1var": ("C1var", dict()),
    "C2x64": ("C2", dict(streams=64)),
    "C2": ("C2", dict(hash_data=0)),
    "C3": ("C3", dict()),
    "C4x256": ("C4", dict(streams=256)),
    "C4": ("C4", dict(hash_data=0)),
    "C5x2000": ("C5", dict(originals=2000)),
    "C5": ("C5", dict(hash_data=0)),
    # full-size configs with every byte of every recovery packet and
    # recovered original hashed (the bench legs' and the headline shard's
    # exact workloads)
    "C2h": ("C2", dict(hash_data=1)),
    "C4x1024h": ("C4", dict(streams=1024, hash_data=1)),
    "C5h": ("C5", dict(hash_data=1)),
    # edge cases: tiny packets, variable sizes in block mode, heavy loss with
    # decode failures / stalls, losses close to the 255-column solver limit,
    # lag-based acknowledgements over a long variable-size stream
    "edge_tiny": ("C2", dict(streams=32, payload_bytes=1, loss_pct=15, recovery_loss_pct=15)),
    "edge_var_block": ("C4", dict(streams=32, originals=300, payload_bytes=0, loss_pct=30,
                                  recovery_loss_pct=10)),
    "edge_heavy": ("C3", dict(originals=3000, loss_pct=40, recovery_loss_pct=40,
                              recovery_interval=2)),
    "edge_maxloss": ("C4", dict(streams=4, originals=1000, loss_pct=24, recovery_loss_pct=0,
                                tail_limit=400)),
    "edge_lag": ("C1", dict(originals=2000, payload_bytes=0, streams=2)),
    # block mode with the originals added by range calls (harness
    # Stream::add_ranges; the reference runs the same sequence as loops of
    # its single calls): the headline shard as bench.py runs it, every byte
    # hashed, and variable sizes
    "smoke_C4x8r": ("C4", dict(streams=8, add_ranges=1)),
    "C4x1024hr": ("C4", dict(streams=1024, hash_data=1, add_ranges=1)),
    "C4r": ("C4", dict(hash_data=0, add_ranges=1)),
    "edge_var_block_r": ("C4", dict(streams=32, originals=300, payload_bytes=0, loss_pct=30,
                                    recovery_loss_pct=10, add_ranges=1)),
    # interleaved configs with range calls: the originals up to each encode
    # point in one call, one acknowledgement per encode interval (the C2 leg
    # as bench.py runs it, every byte hashed; lag-based acks; variable sizes)
    "C2hr": ("C2", dict(hash_data=1, add_ranges=1)),
    "C2x64r": ("C2", dict(streams=64, add_ranges=1)),
    "C1r": ("C1", dict(add_ranges=1, streams=8)),
    "C1var_r": ("C1var", dict(add_ranges=1)),
}


def config(name):
    base, over = FIXTURES[name]
    return S.replace(S.CONFIGS[base], **over)


def path(name):
    return os.path.join(DIR, name + ".json")


def load(name):
    with open(path(name)) as f:
        return json.load(f)


def save(name, cfg, results, seconds):
    data = {
        "name": name,
        "generator": "tests/golden/make_golden.py (oracle/_ref/libsiamese_ref.so)",
        "config": cfg.as_dict(),
        "digests": S.digests(results),
        "status": [int(r.status) for r in results],
        "summary": S.summary(results),
        "reference_seconds": round(seconds, 3),
    }
    with open(path(name), "w") as f:
        json.dump(data, f, separators=(",", ":"))
