"""ctypes front-end of harness/libscenario.so (the loopback workload driver).

Test infrastructure: used by tests/, bench.py (cpu_baseline leg and the GPU
leg) and __graft_entry__.smoke().  It drives any siamese.h implementation --
the upstream reference compiled into oracle/_ref/, the drop-in API of
siamese_amd/libsiamese_amd.so, or the test-only host simulation -- through
the same deterministic call sequence and returns per-stream event digests.
"""
import ctypes
import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENARIO_LIB = os.path.join(ROOT, "harness", "libscenario.so")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libsiamese_ref.so")
REF_COUNTED_LIB = os.path.join(ROOT, "oracle", "_ref", "libsiamese_ref_counted.so")
AMD_LIB = os.path.join(ROOT, "siamese_amd", "libsiamese_amd.so")
SIM_LIB = os.path.join(ROOT, "tests", "hostsim", "libsiamese_hostsim.so")

_FIELDS = ("block_mode streams first_stream originals payload_bytes loss_pct "
           "recovery_loss_pct recovery_interval recovery_phase ack_policy ack_lag "
           "tail_limit seed hash_data add_ranges").split()


class Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in _FIELDS]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in _FIELDS}


class StreamResult(ctypes.Structure):
    _fields_ = ([("digest", ctypes.c_uint64), ("recovery_bytes", ctypes.c_uint64),
                 ("payload_bytes", ctypes.c_uint64)] +
                [(n, ctypes.c_uint32) for n in
                 "encodes recovery_lost originals_lost recovered decode_calls "
                 "decode_fail delivered status".split()])


def make_config(**kw):
    base = dict(block_mode=0, streams=1, first_stream=0, originals=200, payload_bytes=1400,
                loss_pct=10, recovery_loss_pct=5, recovery_interval=8, recovery_phase=0,
                ack_policy=0, ack_lag=40, tail_limit=600, seed=1013, hash_data=1, add_ranges=0)
    base.update(kw)
    return Config(**base)


# Workloads of BASELINE.json / SURVEY.md section 8(d).  `streams` is the
# full size; tests scale it down with replace().
CONFIGS = {
    # C1: reference StreamingTest semantics, 200 x 1400 B, 10% loss
    "C1": make_config(originals=200, loss_pct=10, recovery_loss_pct=5, recovery_interval=8,
                      ack_policy=2, ack_lag=40),
    # C1 with the reference's variable packet sizes 2..1199 B
    "C1var": make_config(originals=300, payload_bytes=0, loss_pct=10, recovery_loss_pct=5,
                         recovery_interval=8, ack_policy=2, ack_lag=40, streams=4),
    # C2: 1024 streams x 256 x 1400 B, 10% loss, 1-in-8, immediate ack (Cauchy path)
    "C2": make_config(streams=1024, originals=256, loss_pct=10, recovery_loss_pct=10,
                      recovery_interval=8, ack_policy=1),
    # C3: single stream 8192 x 1400 B, 20% loss, 1-in-3, no acks (Siamese path)
    "C3": make_config(originals=8192, loss_pct=20, recovery_loss_pct=20, recovery_interval=3),
    # C4: 8192 streams x 256 x 1400 B, 20% loss, block mode
    "C4": make_config(block_mode=1, streams=8192, originals=256, loss_pct=20,
                      recovery_loss_pct=20),
    # C5: 16000 x 65536 B, 5% loss, 1-in-10, no acks
    "C5": make_config(originals=16000, payload_bytes=65536, loss_pct=5, recovery_loss_pct=5,
                      recovery_interval=10),
}


def replace(cfg, **kw):
    d = cfg.as_dict()
    d.update(kw)
    return Config(**d)


class BatchOptions(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_uint32), ("warmup", ctypes.c_uint32),
                ("verify", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("threads", ctypes.c_uint32), ("groups", ctypes.c_uint32),
                ("e2e", ctypes.c_uint32), ("digest", ctypes.c_uint32), ("defer", ctypes.c_uint32),
                ("frames", ctypes.c_uint32), ("no_timing", ctypes.c_uint32),
                ("device_ge", ctypes.c_uint32), ("unique", ctypes.c_uint32)]


class BatchReport(ctypes.Structure):
    _fields_ = [("seconds", ctypes.c_double), ("device_ms", ctypes.c_double),
                ("exec_ms", ctypes.c_double), ("setup_seconds", ctypes.c_double),
                ("rounds", ctypes.c_uint64), ("engine", ctypes.c_uint64 * 21),
                ("checked", ctypes.c_uint64), ("mismatches", ctypes.c_uint64),
                ("phase_seconds", ctypes.c_double * 5), ("payload_bytes", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double * 5)]

KERNELS = ("k_ingest", "k_exec", "k_ldpc", "k_solve", "k_ge")

PHASES = ("create", "step", "flush", "resolve", "finish")


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(SCENARIO_LIB)
        _lib.scenario_run_capi.restype = ctypes.c_int
        _lib.scenario_run_capi.argtypes = [ctypes.c_char_p, ctypes.POINTER(Config),
                                           ctypes.POINTER(StreamResult), ctypes.c_uint,
                                           ctypes.POINTER(ctypes.c_double), ctypes.c_char_p]
        _lib.scenario_run_batch.restype = ctypes.c_int
        _lib.scenario_run_batch.argtypes = [ctypes.c_char_p, ctypes.POINTER(Config),
                                            ctypes.POINTER(StreamResult),
                                            ctypes.POINTER(BatchOptions),
                                            ctypes.POINTER(BatchReport)]
    return _lib


def run_capi(library, cfg, threads=1, event_log=None):
    """Run `cfg` through the siamese.h API of `library`.

    Returns (results array, codec seconds, wall seconds).  Codec seconds: the
    time spent inside codec calls (one thread), or the longest any thread
    spent inside them (several threads, each driving its own streams
    concurrently); payload generation and checking are outside it."""
    res = (StreamResult * cfg.streams)()
    sec = ctypes.c_double()
    t0 = time.time()
    rc = lib().scenario_run_capi(library.encode(), ctypes.byref(cfg), res, threads,
                                 ctypes.byref(sec), event_log.encode() if event_log else None)
    wall = time.time() - t0
    if rc != 0:
        raise RuntimeError("scenario_run_capi(%s) failed rc=%d" % (library, rc))
    return res, sec.value, wall


def run_batch(library, cfg, steps=1, warmup=0, verify=True, device=-1, threads=0, groups=1,
              e2e=False, defer=0, frames=False, device_ge=False, unique=False):
    """Run `cfg` through the device-resident batch API (lock-step rounds),
    streams driven by `threads` host threads (0 = library default), split
    into `groups` groups whose host work and device work alternate.  With
    e2e the originals are copied from pinned host memory every step and every
    recovery packet and recovered original is copied back.  defer=k > 0: the
    deferred-output API, a stream yields after every k-th decode and a group
    keeps up to two submissions in flight.  frames (with e2e): packets travel
    as framed datagrams (sgpu_frames_recv / sgpu_frames_send).  device_ge
    (defer=0): decodes by sgpu_decode_device (the recovery matrix generated
    and eliminated on the device).

    Returns (results of the last run, BatchReport)."""
    res = (StreamResult * cfg.streams)()
    opt = BatchOptions(steps, warmup, 1 if verify else 0, device, threads, groups, 1 if e2e else 0, 1, defer,
                       1 if frames else 0, 0, 1 if device_ge else 0, 1 if unique else 0)
    rep = BatchReport()
    rc = lib().scenario_run_batch(library.encode(), ctypes.byref(cfg), res, ctypes.byref(opt),
                                  ctypes.byref(rep))
    if rc != 0:
        raise RuntimeError("scenario_run_batch(%s) failed rc=%d" % (library, rc))
    return res, rep


ENGINE_KEYS = ("flushes launches ops terms solves ingests upload_bytes ref_op_bytes "
               "out_bytes solve_bytes assemble_ns wait_ns complete_ns reclaim_ns "
               "exec_launches ldpc_bytes exec_unique_bytes ge_jobs ge_chained ge_retried "
               "arena_growth").split()


def engine_dict(report):
    return {k: int(report.engine[i]) for i, k in enumerate(ENGINE_KEYS)}


class BatchSession:
    """Payloads staged in HBM once; run() repeats the workload (bench.py)."""

    def __init__(self, library, cfg, device=-1):
        L = lib()
        L.scenario_batch_open.restype = ctypes.c_void_p
        L.scenario_batch_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(Config), ctypes.c_int]
        L.scenario_batch_run.restype = ctypes.c_int
        L.scenario_batch_run.argtypes = [ctypes.c_void_p, ctypes.POINTER(StreamResult),
                                         ctypes.POINTER(BatchOptions),
                                         ctypes.POINTER(BatchReport)]
        L.scenario_batch_close.argtypes = [ctypes.c_void_p]
        self.cfg = cfg
        self.handle = L.scenario_batch_open(library.encode(), ctypes.byref(cfg), device)
        if not self.handle:
            raise RuntimeError("scenario_batch_open(%s) failed" % library)

    def run(self, steps=1, warmup=0, verify=False, threads=0, groups=1, e2e=False, digest=True, defer=0,
            frames=False, timing=True, device_ge=False, unique=False):
        """digest=False: timed runs skip the per-stream event logs (results
        then carry no digest; take it from a verified run).  device_ge (with
        defer=0): decodes by sgpu_decode_device.  unique: count the executor
        launches' compulsory bytes (sgpu_measure_unique; a measurement run)."""
        res = (StreamResult * self.cfg.streams)()
        opt = BatchOptions(steps, warmup, 1 if verify else 0, -1, threads, groups,
                           1 if e2e else 0, 1 if digest else 0, defer, 1 if frames else 0,
                           0 if timing else 1, 1 if device_ge else 0, 1 if unique else 0)
        rep = BatchReport()
        rc = lib().scenario_batch_run(self.handle, res, ctypes.byref(opt), ctypes.byref(rep))
        if rc != 0:
            raise RuntimeError("scenario_batch_run failed rc=%d" % rc)
        return res, rep

    def close(self):
        if self.handle:
            lib().scenario_batch_close(self.handle)
            self.handle = None


def digests(results):
    return [int(r.digest) for r in results]


def summary(results):
    keys = ("encodes recovery_lost originals_lost recovered decode_calls decode_fail "
            "delivered").split()
    out = {k: int(sum(getattr(r, k) for r in results)) for k in keys}
    out["payload_bytes"] = int(sum(r.payload_bytes for r in results))
    out["recovery_bytes"] = int(sum(r.recovery_bytes for r in results))
    st = [int(r.status) for r in results]
    out["status"] = {str(s): st.count(s) for s in sorted(set(st))}
    return out
