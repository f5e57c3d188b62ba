#!/usr/bin/env python3
"""bench.py -- device-resident encode+decode throughput of the MI355X
streaming erasure codec (BASELINE.json metric), one JSON line on rank 0.

Workload (per GPU, weak scaling): the C4 shard -- 1024 independent streams x
256 originals x 1400 B, 20% loss on originals and recovery packets, block
mode (all originals added, then recovery packets until every original is
delivered).  8 GPUs x 1024 streams = C4's 8192 streams; rank r runs global
streams [1024 r, 1024 (r+1)), so no data-path collective exists.

A "step" is that whole workload: create 1024 encoder/decoder pairs, ingest
the originals (already resident in HBM), encode, drop, decode, free.  The
timed region covers the full step: host control plane and device work.

value  = algorithmic bytes / step time, summed over ranks (GB/s): the source
         bytes of every GF(256) add/mul/muladd the reference codec performs
         for the same call sequence, plus the recovery packets and recovered
         originals written (counted by the library).
roofline = the executor kernel k_exec: the bytes it must move per launch (the
         physical HBM traffic of a committed rocprofv3 PMC capture of this
         build, else the compulsory bytes the library counts) over its
         average launch time (HIP events on the codec's stream), against the
         8 TB/s HBM3E peak.
cpu_baseline = the upstream reference (oracle/_ref, built from
         /root/reference's own sources) on the host cores, same workload on a
         bounded sample of streams.
legs   = (N=1 only) the other BASELINE configs on one GPU -- C2 (1024 streams,
         Cauchy/parity path), C3 (one 8192-packet stream) and C5 (one stream of
         16000 x 64 KiB) -- each with the reference on the host cores beside it.

Multi-GPU: `bench.py --gpus N` (no WORLD_SIZE in the environment) starts N
rank processes itself, one per GPU, from a parent that never touches the GPU;
under torch.distributed.run the ranks come from the environment.  Barrier and
max/sum reductions use gloo on the host: no RCCL anywhere (there is no
data-path exchange between stream shards).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import scenario_lib as S  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
STREAMS_PER_GPU = 1024
METRIC = "device-resident GB/s encode+decode, 1400B pkts @20% loss; % HBM peak"

TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r6_traffic.json")


def lib_sha256(path):
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def pmc_traffic(kernel, library):
    """Per-launch memory traffic of `kernel` from the committed PMC capture
    (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per dispatch, tools/pmc_traffic.py),
    whether that capture measured the very library this run loads (sha256 of
    the .so recorded at capture time), and the capture's traffic of all the
    library's kernels per workload step (None if it has none)."""
    try:
        with open(TRAFFIC_JSON) as f:
            d = json.load(f)
        want = d.get("_lib_sha256")
        same = want is not None and want == lib_sha256(library)
        per_step = None
        if kernel in d.get("_step_dispatches", {}):
            per_step = d[kernel]["traffic_bytes"] * d["_step_dispatches"][kernel]
        return (d[kernel]["traffic_bytes"], d.get("_source", TRAFFIC_JSON), same, d.get("_step_traffic_bytes"),
                per_step)
    except (OSError, KeyError, ValueError):
        return None, None, False, None, None


def workload(rank, streams, ranges=True):
    """The C4 shard of `rank`.  ranges: each stream's originals go to its
    encoder and decoder in range calls (sgpu_encoder_add_range,
    sgpu_decoder_add_original_range, sgpu_decoder_get_range), the same
    data-plane work as the per-packet calls (harness Stream::add_ranges)."""
    return S.replace(S.CONFIGS["C4"], streams=streams, first_stream=rank * streams,
                     hash_data=0, add_ranges=1 if ranges else 0)


def symbol_bytes(payload):
    """Length prefix + payload (reference SiameseSerializers.h:566-593)."""
    return payload + (1 if payload <= 0x7f else 2 if payload <= 0x3fff else 3 if payload <= 0x1fffff else 4)


def ref_algorithmic_bytes(cfg, threads):
    """Algorithmic bytes of `cfg` as the reference itself runs
    it: the source bytes of every bulk GF(256) op, counted by the op-counting
    build of the unmodified reference (oracle/_ref/libsiamese_ref_counted.so),
    plus the recovery packets and recovered originals it writes."""
    if not os.path.exists(S.REF_COUNTED_LIB):
        return None
    lib = ctypes.CDLL(S.REF_COUNTED_LIB)
    lib.ref_op_bytes.restype = ctypes.c_uint64
    lib.ref_op_bytes.argtypes = [ctypes.c_int]
    lib.ref_op_bytes(1)
    res, _, _ = S.run_capi(S.REF_COUNTED_LIB, cfg, threads=threads)
    ops = lib.ref_op_bytes(1)
    if any(r.status for r in res) or cfg.payload_bytes == 0:
        return None
    out = sum(r.recovery_bytes for r in res) + sum(r.recovered for r in res) * symbol_bytes(cfg.payload_bytes)
    return ops + out


def host_info():
    """The host cores the CPU baselines run on."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    return {"nproc": os.cpu_count(), "usable_cpus": usable, "cpu_model": model}


def cgroup_cpu():
    """(process CPU seconds, cgroup throttled seconds or None): read around
    the timed region to tell whether the step is held by the box's CPU quota
    (cgroup v2 cpu.stat of this process's cgroup)."""
    t = os.times()
    cpu = t.user + t.system
    throttled = None
    try:
        with open("/proc/self/cgroup") as f:
            rel = [l.split("::", 1)[1].strip() for l in f if l.startswith("0::")]
        for base in (("/sys/fs/cgroup" + rel[0]) if rel else None, "/sys/fs/cgroup"):
            if not base:
                continue
            p = os.path.join(base, "cpu.stat")
            if os.path.exists(p):
                with open(p) as f:
                    kv = dict(l.split() for l in f if len(l.split()) == 2)
                throttled = int(kv.get("throttled_usec", 0)) / 1e6
                break
    except (OSError, ValueError, IndexError):
        pass
    return cpu, throttled


def thread_cpu():
    """CPU nanoseconds per thread name (/proc/self/task/*/schedstat): the
    library names its threads (sgpu-step, sgpu-assemble, sgpu-launch,
    sgpu-complete); the rest are the process's own."""
    out = {}
    base = "/proc/self/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for t in tids:
        try:
            with open(os.path.join(base, t, "comm")) as f:
                name = f.read().strip()
            with open(os.path.join(base, t, "schedstat")) as f:
                ns = int(f.read().split()[0])
        except (OSError, ValueError, IndexError):
            continue
        if not name.startswith("sgpu-"):
            name = "other"
        out[name] = out.get(name, 0) + ns
    return out


def cgroup_quota():
    """The cgroup's CPU quota in CPUs (cpu.max), or None."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = [l.split("::", 1)[1].strip() for l in f if l.startswith("0::")]
        for base in (("/sys/fs/cgroup" + rel[0]) if rel else None, "/sys/fs/cgroup"):
            if base and os.path.exists(os.path.join(base, "cpu.max")):
                with open(os.path.join(base, "cpu.max")) as f:
                    q, per = f.read().split()[:2]
                return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError, IndexError):
        pass
    return None


class CpuBaseline:
    """The reference codec on `threads` host cores over `cfg` (a bounded
    sample of the workload), measured once per measure() call so the runs can
    be interleaved with the GPU runs they are compared to.  A run's value =
    the reference's own algorithmic bytes for exactly this sample
    (op-counting build, one untimed run) over the time spent inside codec
    calls (the longest thread's, when several drive their own streams at
    once); payload generation is not timed.  The reported value is the
    median run."""

    def __init__(self, cfg, threads, sample):
        self.cfg, self.threads, self.sample = cfg, threads, sample
        self.alg = ref_algorithmic_bytes(cfg, threads) if os.path.exists(S.REF_LIB) else None
        self.runs = []   # (GB/s, codec seconds, wall seconds, payload bytes)

    def measure(self):
        if self.alg is None:
            return None
        res, sec, wall = S.run_capi(S.REF_LIB, self.cfg, threads=self.threads)
        if sec <= 0 or any(r.status for r in res):
            return None
        v = self.alg / sec / 1e9
        self.runs.append((v, sec, wall, sum(r.payload_bytes for r in res)))
        return v

    def result(self, gpu_values=None):
        """gpu_values: the GPU run beside each CPU run (same order), for
        per-run ratios."""
        if not self.runs:
            return None
        order = sorted(range(len(self.runs)), key=lambda i: self.runs[i][0])
        v, sec, wall, payload = self.runs[order[len(order) // 2]]
        out = {
            "value": round(v, 3),
            "unit": "GB/s",
            "payload_GBps": round(payload / sec / 1e9, 3),
            "cores": self.threads,
            "kind": "reference",
            "runs_all": [round(r[0], 3) for r in self.runs],
            "sample": "%s on %d thread%s: median of %d runs, %.4f s in codec calls (%.4f s wall), "
                      "%d algorithmic bytes" % (self.sample, self.threads, "s" if self.threads > 1 else "",
                                                len(self.runs), sec, wall, self.alg),
            "host": host_info(),
        }
        if gpu_values:
            ratios = [g / r[0] for g, r in zip(gpu_values, self.runs) if g and r[0]]
            if ratios:
                out["ratio"] = [round(x, 2) for x in ratios]
                out["ratio_median"] = round(sorted(ratios)[len(ratios) // 2], 2)
                out["ratio_note"] = "GPU value / reference value of the runs taken side by side"
        return out


def cpu_baseline(cfg, threads, sample, runs=3):
    """CpuBaseline over `runs` back-to-back runs (no GPU runs beside it)."""
    cb = CpuBaseline(cfg, threads, sample)
    for _ in range(runs):
        cb.measure()
    return cb.result()


class Collective:
    """Barrier + reductions over ranks on the host (gloo), or no-ops at N=1."""

    def __init__(self, world):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            self.dist = dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def reduce(self, values, op):
        if self.dist is None:
            return [float(v) for v in values]
        import torch
        t = torch.tensor(values, dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max"
                             else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.tolist()]

    def close(self):
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()


def engine_bytes(rep):
    eng = S.engine_dict(rep)
    return eng, eng["ref_op_bytes"] + eng["out_bytes"]


def run_leg(name, library, cfg, device, threads, runs, cpu_cfg, cpu_threads, cpu_sample, defer):
    """One extra BASELINE config on one GPU: a verified warm-up, then `runs`
    timed runs ONE AT A TIME (no run overlaps another run of the same
    streams), the median reported; the reference on the host beside it.
    C2's 1024 streams run in four pipelined stream groups (one group's host
    work beside the others' device work: 22.5-24.4 vs 25.0-26.6 ms per run
    with one group against two, profiles/r2l_c2_groups_ab.txt; four against
    two 12.7-13.7 vs 13.2-14.3 ms, round 6, profiles/r6v_c2_groups.txt); a
    single stream is one group.  `defer`: the deferred-output API (siamese_gpu.h),
    a stream submits after every `defer`-th decode and is driven on while
    up to two of its submissions run (profiles/r3c_defer_sweep.txt)."""
    groups = 4 if cfg.streams >= 64 else 1
    cb = CpuBaseline(cpu_cfg, cpu_threads, cpu_sample) if cpu_cfg is not None else None
    sess = S.BatchSession(library, cfg, device=device)
    per = []
    gpu_vals = []
    try:
        res, rep = sess.run(steps=0, warmup=1, verify=True, threads=threads, groups=groups,
                            defer=defer)
        if rep.mismatches or any(r.status for r in res):
            raise RuntimeError("bench leg %s: verification failed" % name)
        # the timed runs without per-launch timing events (each orders its
        # launch behind a timestamp: +30 % on C3, profiles/r3f_timing_ab.txt),
        # each followed by a run of the reference on the host (interleaved,
        # so both see the same box), then one more GPU run with the events
        # for the device and per-kernel times
        for _ in range(runs):
            res, rep = sess.run(steps=1, warmup=0, verify=False, threads=threads, groups=groups,
                                digest=False, defer=defer, timing=False)
            per.append(rep)
            if cb is not None:
                _, a = engine_bytes(rep)
                gpu_vals.append(a / rep.seconds / 1e9)
                cb.measure()
        _, trep = sess.run(steps=1, warmup=0, verify=False, threads=threads, groups=groups,
                           digest=False, defer=defer, timing=True)
    finally:
        sess.close()
    order = sorted(range(len(per)), key=lambda i: per[i].seconds)
    rep = per[order[len(order) // 2]]   # the median run
    eng, alg = engine_bytes(rep)
    teng, talg = engine_bytes(trep)
    payload = rep.payload_bytes   # (one run)
    sec = rep.seconds
    kms = dict(zip(S.KERNELS, trep.kernel_ms))
    exec_s = kms["k_exec"] / 1e3
    ldpc_s = kms["k_ldpc"] / 1e3
    exec_bytes = talg - teng["solve_bytes"] - teng["ldpc_bytes"]
    ldpc_bytes = teng["ldpc_bytes"]
    out = {
        "workload": "%d stream%s x %d originals x %d B, %d%% loss" % (
            cfg.streams, "s" if cfg.streams > 1 else "", cfg.originals, cfg.payload_bytes,
            cfg.loss_pct),
        "add_calls": "range (up to each encode point)" if cfg.add_ranges else "per packet",
        "runs": runs,
        "stream_groups": groups,
        "defer": defer,
        "ms_per_run": round(sec * 1e3, 3),
        "ms_per_run_all": [round(r.seconds * 1e3, 3) for r in per],
        "value": round(alg / sec / 1e9, 3),
        "unit": "GB/s",
        "payload_GBps": round(payload / sec / 1e9, 3),
        "device_ms_per_run": round(trep.device_ms, 3),
        "kernel_ms_per_run": {k: round(v, 3) for k, v in kms.items()},
        "device_ms_note": "one extra run with per-launch HIP events (the timed runs have none)",
        "rounds_per_run": rep.rounds,
        "algorithmic_bytes_per_run": alg,
        "payload_bytes_per_run": payload,
        "roofline": {
            "bound": "hbm", "kernel": "k_exec",
            "achieved": round(exec_bytes / exec_s / 1e9, 2) if exec_s > 0 else None,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(exec_bytes / exec_s / 1e9 / HBM_PEAK_GBPS, 4) if exec_s > 0 else None,
            "bytes_per_run": exec_bytes,
        },
        "roofline_ldpc": {
            "bound": "hbm", "kernel": "k_ldpc",
            "achieved": round(ldpc_bytes / ldpc_s / 1e9, 2) if ldpc_s > 0 else None,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ldpc_bytes / ldpc_s / 1e9 / HBM_PEAK_GBPS, 4) if ldpc_s > 0 else None,
            "bytes_per_run": ldpc_bytes,
        } if ldpc_bytes else None,
        "cpu_baseline": None,
    }
    if cb is not None:
        out["cpu_baseline"] = cb.result(gpu_vals)
    return out


def dropin_leg(library, use_cpu, runs=5):
    """C1 through the drop-in siamese.h ABI: one stream, every call
    synchronous with its own flush, as a caller of the reference API sees it
    (latency per call, not throughput).  The reference on one core beside it."""
    cfg = S.replace(S.CONFIGS["C1"], hash_data=0)

    def measure(lib):
        S.run_capi(lib, cfg)   # warm
        wall = codec = 0.0
        calls = 0
        for _ in range(runs):
            res, sec, w = S.run_capi(lib, cfg)
            if any(r.status for r in res):
                raise RuntimeError("drop-in leg: stream failed (%s)" % lib)
            wall += w
            codec += sec
            for r in res:
                # encoder adds + decoder adds, encodes + recovery adds,
                # decodes, in-order deliveries (get)
                calls += (2 * cfg.originals - r.originals_lost + 2 * r.encodes - r.recovery_lost +
                          r.decode_calls + r.delivered)
        return {"ms_per_run": round(wall / runs * 1e3, 3),
                "codec_ms_per_run": round(codec / runs * 1e3, 3),
                "calls_per_run": calls // runs,
                "us_per_call": round(codec / max(1, calls) * 1e6, 3)}

    out = {"workload": "C1 through siamese.h (1 stream x 200 x 1400 B, 10% loss, acks)", "runs": runs}
    out.update(measure(library))
    out["cpu_baseline"] = None
    if use_cpu and os.path.exists(S.REF_LIB):
        ref = measure(S.REF_LIB)
        ref.update({"cores": 1, "kind": "reference"})
        out["cpu_baseline"] = ref
    return out


def dropin_threads_leg(library, use_cpu, threads=16, runs=3):
    """C2 through the drop-in siamese.h ABI from `threads` application
    threads at once, each driving its own 1024/threads streams (per-instance
    calls concurrent, flushes group-committed), every stream's digest
    checked against the reference's own run of the same streams; the
    reference on the same number of threads beside it (interleaved runs)."""
    cfg = S.replace(S.CONFIGS["C2"], hash_data=0)
    alg = ref_algorithmic_bytes(cfg, threads) if use_cpu else None
    gpu, ref = [], []
    ref_digests = None
    for _ in range(runs):
        res, sec, wall = S.run_capi(library, cfg, threads=threads)
        if any(r.status for r in res):
            raise RuntimeError("drop-in C2 leg: a stream failed")
        gpu.append((sec, wall, S.digests(res)))
        if use_cpu and os.path.exists(S.REF_LIB):
            rres, rsec, rwall = S.run_capi(S.REF_LIB, cfg, threads=threads)
            ref.append((rsec, rwall))
            ref_digests = S.digests(rres)
    if ref_digests is not None and any(g[2] != ref_digests for g in gpu):
        raise RuntimeError("drop-in C2 leg: digests differ from the reference's")
    walls = sorted(g[1] for g in gpu)
    out = {"workload": "C2 through siamese.h from %d threads (%d streams each)" % (threads, cfg.streams // threads),
           "runs": runs, "threads": threads,
           "wall_ms_all": [round(g[1] * 1e3, 3) for g in gpu],
           "wall_ms": round(walls[len(walls) // 2] * 1e3, 3),
           "digests_match_reference": ref_digests is not None,
           "cpu_baseline": None}
    if alg:
        out["value"] = round(alg / walls[len(walls) // 2] / 1e9, 3)
        out["unit"] = "GB/s (reference algorithmic bytes / wall time)"
    if ref:
        rw = sorted(r[1] for r in ref)
        out["cpu_baseline"] = {"wall_ms_all": [round(r[1] * 1e3, 3) for r in ref],
                               "wall_ms": round(rw[len(rw) // 2] * 1e3, 3), "cores": threads,
                               "kind": "reference",
                               "value": round(alg / rw[len(rw) // 2] / 1e9, 3) if alg else None,
                               "ratio_median": round(rw[len(rw) // 2] / walls[len(walls) // 2], 2)}
    return out


def legs(library, device, threads, use_cpu):
    cpu_threads = min(16, host_info()["usable_cpus"] or 1)
    specs = [
        # C2: 1024 streams, Cauchy/parity path; reference on all host cores.
        # Per-packet calls: range calls up to each encode point (fixture
        # C2hr) measured the same wall time (13.2-14.4 vs 13.7-15.8 ms per
        # run, profiles/r4ak_c2_ranges_ab.txt): a run is bound by its ten
        # rounds' flush-to-completion latency, not by host CPU
        ("C2", S.replace(S.CONFIGS["C2"], hash_data=0), 3,
         S.replace(S.CONFIGS["C2"], hash_data=0), cpu_threads,
         "the full C2 (1024 streams x 256 x 1400 B)", 4),
        # C3: one stream; reference on one core (an instance is single-threaded)
        ("C3", S.replace(S.CONFIGS["C3"], hash_data=0), 3,
         S.replace(S.CONFIGS["C3"], hash_data=0), 1, "the full C3 (1 stream x 8192 x 1400 B)", 8),
        # C5: one stream of 64 KiB symbols; reference on one core over the
        # first 2000 originals (the whole stream takes it ~15 s)
        ("C5", S.replace(S.CONFIGS["C5"], hash_data=0), 3,
         S.replace(S.CONFIGS["C5"], hash_data=0, originals=2000), 1,
         "C5's first 2000 originals (1 stream x 2000 x 64 KiB)", 8),
    ]
    out = {}
    for name, cfg, runs, cpu_cfg, cpu_thr, sample, defer in specs:
        out[name] = run_leg(name, library, cfg, device, threads, runs,
                            cpu_cfg if use_cpu else None, cpu_thr, sample, defer)
    out["dropin_C1"] = dropin_leg(library, use_cpu)
    out["dropin_C2_threads"] = dropin_threads_leg(library, use_cpu, threads=min(16, cpu_threads))
    return out


def run_rank(rank, world, local, args, library, use_cuda):
    """One rank's share: returns the JSON line on rank 0, None elsewhere."""
    coll = Collective(world)
    cfg = workload(rank, args.streams, args.ranges)
    device = local if use_cuda else -1
    sess = S.BatchSession(library, cfg, device=device)
    # untimed warm-up; its first run checks every recovered byte against the payload
    dge = args.device_ge and args.defer == 0
    res, rep = sess.run(steps=0, warmup=1, verify=args.verify, threads=args.threads,
                        groups=args.groups, defer=args.defer, device_ge=dge)
    if args.verify and (rep.mismatches or any(r.status for r in res)):
        raise RuntimeError("bench: verification failed: %d byte mismatches, status %s"
                           % (rep.mismatches, S.summary(res)["status"]))
    # determinism fingerprint of the (verified) workload; the timed steps
    # repeat it exactly but keep no event logs
    verified_digests = S.digests(res)
    # then W untimed steps pipelined exactly like the timed ones, so the
    # buffer arena reaches the timed loop's high-water mark before timing
    if args.warmup > 0:
        sess.run(steps=args.warmup, warmup=0, verify=False, threads=args.threads,
                 groups=args.groups, digest=False, defer=args.defer, device_ge=dge)

    # the reference on the host cores (rank 0 at N=1 only) over a bounded
    # sample of C4 streams, one run before the timed steps, one after them
    # and one after the end-to-end leg (interleaved with the GPU's runs)
    cb = None
    side = []   # GPU values of the short side runs taken beside each CPU run

    def side_run():
        # a few untimed steps of the same workload right beside a CPU run, so
        # each reference run has a GPU run under the same box conditions
        # (cpu_baseline.ratio); never part of `value`
        n = max(3, args.steps // 4)
        t = time.perf_counter()
        _, r = sess.run(steps=n, warmup=0, verify=False, threads=args.threads, groups=args.groups,
                        digest=False, defer=args.defer, device_ge=dge, timing=False)
        side.append(engine_bytes(r)[1] / (time.perf_counter() - t) / 1e9)

    if not args.no_cpu and world == 1:
        threads = min(16, host_info()["usable_cpus"] or 1)
        sample_cfg = S.replace(S.CONFIGS["C4"], streams=args.cpu_streams, first_stream=0,
                               hash_data=0, add_ranges=1 if args.ranges else 0)
        cb = CpuBaseline(sample_cfg, threads, "%d C4 streams (256 x 1400 B, 20%% loss, block mode)"
                         % args.cpu_streams)
        # (the reference's 16-thread runs come after the timed steps: a
        # timed run right behind one measured slower, the host still
        # recovering from the all-core load; --cpu-first keeps the old order)
        if args.cpu_first:
            cb.measure()
            side_run()

    coll.barrier()
    cpu0, thr0 = cgroup_cpu()
    th0 = thread_cpu()
    t0 = time.perf_counter()
    res, rep = sess.run(steps=args.steps, warmup=0, verify=False, threads=args.threads,
                        groups=args.groups, digest=False, defer=args.defer, device_ge=dge)
    coll.barrier()
    elapsed = time.perf_counter() - t0
    cpu1, thr1 = cgroup_cpu()
    th1 = thread_cpu()
    cpu_used = {"process_cpus": round((cpu1 - cpu0) / elapsed, 2),
                "cpu_ms_per_step_by_thread": {k: round((th1[k] - th0.get(k, 0)) / 1e6 / args.steps, 3)
                                              for k in sorted(th1)},
                "cgroup_quota_cpus": cgroup_quota(),
                "cgroup_throttled_ms": round((thr1 - thr0) * 1e3, 2) if thr0 is not None and thr1 is not None
                else None}
    # one untimed step that counts the executor's compulsory bytes (every
    # distinct symbol read once, every output written once: the roofline's
    # byte figure; counting it costs assembly time, so never in the timed run)
    _, urep = sess.run(steps=1, warmup=0, verify=False, threads=args.threads, groups=args.groups,
                       digest=False, defer=args.defer, device_ge=dge, unique=True)
    # the same steps with the other placement of the coefficient elimination
    # (host / device), timed the same way right after: reported beside
    # `value`, never as it
    alt_elapsed = None
    if args.decode_ab and args.defer == 0:
        sess.run(steps=max(1, args.warmup), warmup=0, verify=False, threads=args.threads, groups=args.groups,
                 digest=False, defer=args.defer, device_ge=not dge)
        coll.barrier()
        ta = time.perf_counter()
        sess.run(steps=args.steps, warmup=0, verify=False, threads=args.threads, groups=args.groups,
                 digest=False, defer=args.defer, device_ge=not dge, timing=False)
        coll.barrier()
        alt_elapsed = time.perf_counter() - ta
    if cb is not None:
        cb.measure()
        side_run()
        if not args.cpu_first:
            cb.measure()
            side_run()

    # End-to-end (PCIe-inclusive) leg, timed separately: the originals start
    # in pinned host memory and every recovery packet and recovered original
    # is copied back to the host (originals delivered intact are not: the
    # application holds them in host memory already).  Reported beside, never
    # as, `value`.
    e2e_elapsed = None
    if args.e2e:
        # (pipelined warm-up over both alternating device copies, every
        # recovered byte checked against the payloads)
        res_e, rep_e = sess.run(steps=max(2, args.warmup), warmup=0, verify=args.verify,
                                threads=args.threads, groups=args.groups, e2e=True, digest=False, defer=args.defer,
                                frames=args.frames, device_ge=dge)
        if args.verify and (rep_e.mismatches or any(r.status for r in res_e)):
            raise RuntimeError("bench: end-to-end verification failed: %d byte mismatches"
                               % rep_e.mismatches)
        coll.barrier()
        t1 = time.perf_counter()
        sess.run(steps=args.steps, warmup=0, verify=False, threads=args.threads,
                 groups=args.groups, e2e=True, digest=False, defer=args.defer, frames=args.frames, device_ge=dge)
        coll.barrier()
        e2e_elapsed = time.perf_counter() - t1
    if cb is not None:
        cb.measure()
        side_run()
    sess.close()

    eng, alg_bytes = engine_bytes(rep)
    payload = rep.payload_bytes   # (all timed steps)
    digest = 0
    for d in verified_digests:
        digest = (digest * 1099511628211 + d) % (1 << 61)
    t_max, = coll.reduce([elapsed], "max")
    alg_total, payload_total, streams_total = coll.reduce(
        [float(alg_bytes), float(payload), float(cfg.streams)], "sum")
    e2e_max = coll.reduce([e2e_elapsed], "max")[0] if e2e_elapsed is not None else None
    alt_max = coll.reduce([alt_elapsed], "max")[0] if alt_elapsed is not None else None
    extra = None
    if rank == 0 and world == 1 and args.legs:
        extra = legs(library, device, args.threads, not args.no_cpu)
    coll.barrier()
    coll.close()
    if rank != 0:
        return None

    value = alg_total / t_max / 1e9
    exec_s = rep.exec_ms / 1e3
    exec_bytes = alg_bytes - eng["solve_bytes"]
    achieved_alg = (exec_bytes / exec_s / 1e9) if exec_s > 0 else 0.0
    steps = args.steps
    launches = max(1, eng["exec_launches"])
    traffic_capture, traffic_src, traffic_same, step_traffic, exec_traffic_step = pmc_traffic("sgpu::k_exec", library)
    exec_ms_per_launch = rep.exec_ms / launches
    # The capture's per-dispatch average comes from short runs whose pipeline
    # fills and drains every step (more, emptier launches: 17.5 per step there
    # against 16 in a long timed loop); the kernel's traffic PER STEP is the
    # same work either way, so a launch of this run carries the capture's
    # per-step traffic over this run's launches per step.
    traffic = traffic_capture
    if exec_traffic_step and steps:
        traffic = exec_traffic_step / (eng["exec_launches"] / steps)
    ueng = S.engine_dict(urep)
    unique_per_launch = ueng["exec_unique_bytes"] / max(1, ueng["exec_launches"])
    t_launch = exec_ms_per_launch / 1e3
    unique_gbps = unique_per_launch / t_launch / 1e9 if t_launch > 0 else 0.0
    traffic_gbps = traffic / t_launch / 1e9 if traffic and t_launch > 0 else None
    # the roofline's bytes: the physical HBM traffic of this very build when
    # a PMC capture of it is committed, the compulsory bytes otherwise
    phys = traffic_gbps is not None and traffic_same
    achieved = traffic_gbps if phys else unique_gbps
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (reference unit_test SetPacket payloads, PCG loss channel seed 1013)",
        "config": {
            "workload": "C4 shard per GPU: %d streams x 256 originals x 1400 B, 20%% loss, "
                        "block mode, no RCCL" % args.streams,
            "streams_per_gpu": args.streams,
            "streams_total": int(streams_total),
            "originals": 256,
            "payload_bytes": 1400,
            "loss_pct": 20,
            "add_calls": "range (sgpu_encoder_add_range / sgpu_decoder_add_original_range)"
                         if args.ranges else "per packet",
            "decode": "sgpu_decode_device (recovery matrix generated and eliminated on the GPU by k_ge, "
                      "chained with the elimination of received data and the solve into one submission)"
                      if dge else "sgpu_decode (recovery matrix on the host)",
            "parallelism": "independent streams sharded by index (weak scaling), "
                           "one process per GPU, gloo host barrier",
        },
        "decode_ab": ({
            "sgpu_decode_device_ms_per_step": round((t_max if dge else alt_max) / steps * 1e3, 3),
            "sgpu_decode_ms_per_step": round((alt_max if dge else t_max) / steps * 1e3, 3),
            "note": "the same workload and steps with the coefficient elimination on the device "
                    "(GenerateMatrix + GaussianElimination in k_ge, chained into the decode's submission) "
                    "and on the host, timed back to back in this run; `value` is the first",
        } if alt_max is not None else None),
        "payload_GBps": round(payload_total / t_max / 1e9, 3),
        "pct_hbm_peak": round(100.0 * value / (HBM_PEAK_GBPS * world), 2),
        "pct_hbm_peak_basis": "ALGORITHMIC bytes (SURVEY 8d: every source byte of the reference's GF ops, "
                              "re-reads included) over wall time; the memory traffic the step moves is "
                              "physical_step below",
        "physical_step": ({
            "traffic_bytes_per_step": step_traffic,
            "GBps": round(step_traffic * world / t_max * steps / 1e9, 3),
            "pct_hbm_peak": round(100.0 * step_traffic * world / t_max * steps / 1e9
                                  / (HBM_PEAK_GBPS * world), 2),
            "build_matches": traffic_same,
            "note": "all kernels' rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per workload step from the "
                    "committed capture (traffic_source; L2 <-> fabric bytes, MALL hits included) over "
                    "this run's wall time per step",
        } if step_traffic else None),
        "device": {
            "exec_ms_per_step": round(rep.exec_ms / steps, 3),
            "kernel_ms_per_step": {k: round(v / steps, 3) for k, v in zip(S.KERNELS, rep.kernel_ms)},
            "device_ms_per_step": round(rep.device_ms / steps, 3),
            "rounds_per_step": rep.rounds / steps,
            "launches_per_step": eng["launches"] / steps,
            "algorithmic_bytes_per_step": alg_bytes // steps,
            "upload_bytes_per_step": eng["upload_bytes"] // steps,
            "arena_growth_bytes": eng["arena_growth"],
            "rank0_digest": digest,
        },
        "host": {
            "threads": args.threads or "default",
            "groups": args.groups,
            "phase_ms_per_step": {k: round(v * 1e3 / steps, 3)
                                  for k, v in zip(S.PHASES, rep.phase_seconds)},
            "engine_ms_per_step": {k[:-3]: round(eng[k] / 1e6 / steps, 3)
                                   for k in ("assemble_ns", "wait_ns", "complete_ns",
                                             "reclaim_ns")},
            "timed_region_cpu": cpu_used,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_exec",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "frac_basis": ("L2 <-> fabric bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of a "
                           "separate --steps 1 capture of this same library build; MALL hits included, so "
                           "an upper bound on HBM bytes: unique_frac beside it is the compulsory floor)"
                           if phys else "compulsory bytes per launch (no PMC capture of this build committed)"),
            "traffic": round(traffic) if traffic else traffic,
            "traffic_per_capture_dispatch": traffic_capture,
            "traffic_source": traffic_src,
            "traffic_build_matches": traffic_same,
            "traffic_GBps": round(traffic_gbps, 2) if traffic_gbps else None,
            "traffic_frac": round(traffic_gbps / HBM_PEAK_GBPS, 4) if traffic_gbps else None,
            "unique_bytes_per_launch": int(unique_per_launch),
            "unique_GBps": round(unique_gbps, 2),
            "unique_frac": round(unique_gbps / HBM_PEAK_GBPS, 4),
            "exec_ms_per_launch": round(exec_ms_per_launch, 4),
            "exec_launches_per_step": eng["exec_launches"] / steps,
            "achieved_alg": round(achieved_alg, 2),
            "alg_bytes_per_launch": exec_bytes // launches,
            "alg_bytes_per_step": exec_bytes // steps,
            "note": "launch time = k_exec's average HIP-event duration on the codec stream in this run; "
                    "traffic = rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of a committed capture "
                    "(traffic_build_matches: the capture's library sha256 equals this run's), the kernel's "
                    "bytes per workload step there over this run's launches per step "
                    "(traffic_per_capture_dispatch: the capture's own per-dispatch average); unique = "
                    "every distinct symbol read once + every output written once + the op stream, counted "
                    "by the library in one extra untimed step; achieved_alg = SURVEY 8d's ALGORITHMIC "
                    "bytes (every re-read the reference performs) over the same time: NOT a roofline, "
                    "the kernel serves those re-reads from LDS",
        },
        "cpu_baseline": None,
        "end_to_end": None,
        "legs": extra,
    }
    if e2e_max is not None:
        line["end_to_end"] = {
            "value": round(alg_total / e2e_max / 1e9, 3),
            "unit": "GB/s",
            "payload_GBps": round(payload_total / e2e_max / 1e9, 3),
            "ms_per_step": round(e2e_max / steps * 1e3, 3),
            "framed": bool(args.frames),
            "note": "originals H2D from pinned host memory each step%s; every recovery packet "
                    "%sand recovered original D2H, originals delivered intact stay on the host "
                    "(PCIe-inclusive; not `value`)" % (
                        " as framed datagrams handed to the decoders by sgpu_frames_recv"
                        if args.frames else "",
                        "(framed by sgpu_frames_send) " if args.frames else ""),
        }
    if cb is not None:
        line["cpu_baseline"] = cb.result(side)
        if line["cpu_baseline"] is not None:
            line["cpu_baseline"]["ratio_note"] = (
                "GPU/reference per pair: each reference run beside a short untimed GPU run of the same "
                "workload (%d steps), both under the same box conditions" % max(3, args.steps // 4))
    return line


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """Start n rank processes (one per GPU) and wait for them.  The parent
    makes no GPU call; each child binds GPU `LOCAL_RANK` itself."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   SIAMESE_AMD_DEVICE=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    try:
        for p in procs:
            p.wait()
            rc = rc or p.returncode
            if p.returncode:
                for q in procs:
                    if q.poll() is None:
                        q.kill()   # exact PIDs of our own children
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
                q.wait()
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams", type=int, default=STREAMS_PER_GPU)
    ap.add_argument("--cpu-streams", type=int, default=16384)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-first", action="store_true",
                    help="run the first reference measurement before the timed steps (the round-5 order)")
    ap.add_argument("--threads", type=int, default=0,
                    help="host threads driving streams (0 = library default)")
    # (8 since round 6: with the device elimination a group's round carries
    # k_ge and a singular decode's extra round, and smaller groups keep the
    # pipeline fuller: 4.42-4.54 against 4.69-4.77 ms/step with 4, same box,
    # interleaved, profiles/r6g_groups_ab.txt)
    ap.add_argument("--groups", type=int, default=8,
                    help="stream groups alternating host and device work (1 = no overlap)")
    ap.add_argument("--defer", type=int, default=0,
                    help="deferred decode outputs: a stream submits after every DEFER-th decode "
                         "(0: it yields after each decode until its lengths are known)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false",
                    help="skip the PCIe-inclusive end-to-end leg")
    ap.add_argument("--no-frames", dest="frames", action="store_false",
                    help="end-to-end leg with raw payloads instead of framed datagrams")
    ap.add_argument("--device-ge", dest="device_ge", action="store_true", default=True,
                    help="decodes by sgpu_decode_device (recovery matrix on the GPU; the default)")
    ap.add_argument("--no-device-ge", dest="device_ge", action="store_false",
                    help="decodes by sgpu_decode (recovery matrix on the host)")
    ap.add_argument("--no-decode-ab", dest="decode_ab", action="store_false",
                    help="skip the timed run of the other decode placement")
    ap.add_argument("--no-ranges", dest="ranges", action="store_false",
                    help="headline originals through per-packet add/get calls instead of range calls")
    ap.add_argument("--no-legs", dest="legs", action="store_false",
                    help="skip the C2/C3/C5 legs (N=1)")
    ap.add_argument("--library", default=S.AMD_LIB, help=argparse.SUPPRESS)
    # profiling runs over tools/libsiamese_null.so (no symbol work) only
    ap.add_argument("--no-verify", dest="verify", action="store_false", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = os.path.basename(args.library).startswith("libsiamese_amd")
    line = run_rank(rank, world, local, args, args.library, use_cuda)
    if line is not None:
        print(json.dumps(line), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
