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
roofline = the executor kernel k_exec: its share of the algorithmic bytes over
         its summed launch time (HIP events on the codec's stream), against
         the 8 TB/s HBM3E peak.
cpu_baseline = the upstream reference (oracle/_ref, built from
         /root/reference's own sources) on the host cores, same workload on a
         bounded sample of streams.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import scenario_lib as S  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
STREAMS_PER_GPU = 1024
METRIC = "device-resident GB/s encode+decode, 1400B pkts @20% loss; % HBM peak"


TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r1_s8_traffic.json")
TRAFFIC_NOTE = ("HBM bytes per k_exec launch from rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE "
                "of `bench.py --steps 1 --warmup 1 --no-cpu --no-e2e` (profiles/r1_s8_traffic.json, "
                "tools/pmc_traffic.py); compare with exec_bytes_per_launch")


def pmc_traffic(kernel):
    """Per-launch HBM traffic of `kernel` from the committed PMC profile."""
    try:
        with open(TRAFFIC_JSON) as f:
            return json.load(f)[kernel]["traffic_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def workload(rank, streams):
    return S.replace(S.CONFIGS["C4"], streams=streams, first_stream=rank * streams,
                     hash_data=0)


def cpu_baseline(sample_streams, threads, alg_bytes_per_stream):
    """Reference codec on the host cores over a bounded sample of the same workload."""
    if not os.path.exists(S.REF_LIB):
        return None
    cfg = S.replace(S.CONFIGS["C4"], streams=sample_streams, first_stream=0, hash_data=0)
    res, _, wall = S.run_capi(S.REF_LIB, cfg, threads=threads)
    payload = sum(r.payload_bytes for r in res)
    return {
        "value": round(alg_bytes_per_stream * sample_streams / wall / 1e9, 3),
        "unit": "GB/s",
        "payload_GBps": round(payload / wall / 1e9, 3),
        "cores": threads,
        "kind": "reference",
        "sample": "%d C4 streams (256 x 1400 B, 20%% loss, block mode) on %d threads, %.2f s"
                  % (sample_streams, threads, wall),
    }


class Collective:
    """Barrier + reductions over ranks (torch.distributed), or a no-op at N=1."""

    def __init__(self, world, use_cuda):
        import torch
        self.torch = torch
        self.world = world
        self.use_cuda = use_cuda
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            self.dist = dist
            if not dist.is_initialized():
                dist.init_process_group("nccl" if use_cuda else "gloo")

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()
        if self.use_cuda:
            self.torch.cuda.synchronize()

    def reduce(self, values, op):
        t = self.torch.tensor(values, dtype=self.torch.float64,
                              device="cuda" if self.use_cuda else "cpu")
        if self.dist is not None:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max"
                                 else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.tolist()]


def run_rank(rank, world, local, args, library, use_cuda):
    """One rank's share: returns the JSON line on rank 0, None elsewhere."""
    import torch
    if use_cuda:
        torch.cuda.set_device(local)
    coll = Collective(world, use_cuda)
    cfg = workload(rank, args.streams)
    sess = S.BatchSession(library, cfg, device=local if use_cuda else -1)
    # untimed warm-up; its first run checks every recovered byte against the payload
    res, rep = sess.run(steps=0, warmup=max(1, args.warmup), verify=True, threads=args.threads,
                        groups=args.groups)
    if rep.mismatches or any(r.status for r in res):
        raise RuntimeError("bench: verification failed: %d byte mismatches, status %s"
                           % (rep.mismatches, S.summary(res)["status"]))
    # determinism fingerprint of the (verified) workload; the timed steps
    # repeat it exactly but keep no event logs
    verified_digests = S.digests(res)

    coll.barrier()
    t0 = time.perf_counter()
    res, rep = sess.run(steps=args.steps, warmup=0, verify=False, threads=args.threads,
                        groups=args.groups, digest=False)
    coll.barrier()
    elapsed = time.perf_counter() - t0

    # End-to-end (PCIe-inclusive) leg, timed separately: the originals start
    # in pinned host memory and every recovery packet and recovered original
    # is copied back to the host.  Reported beside, never as, `value`.
    e2e_elapsed = None
    if args.e2e:
        sess.run(steps=0, warmup=1, verify=False, threads=args.threads, groups=args.groups,
                 e2e=True)
        coll.barrier()
        t1 = time.perf_counter()
        _, rep_e2e = sess.run(steps=args.steps, warmup=0, verify=False, threads=args.threads,
                              groups=args.groups, e2e=True, digest=False)
        coll.barrier()
        e2e_elapsed = time.perf_counter() - t1
    sess.close()

    eng = S.engine_dict(rep)
    alg_bytes = eng["ref_op_bytes"] + eng["out_bytes"]
    payload = sum(r.payload_bytes for r in res) * args.steps
    digest = 0
    for d in verified_digests:
        digest = (digest * 1099511628211 + d) % (1 << 61)
    t_max, = coll.reduce([elapsed], "max")
    alg_total, payload_total, streams_total = coll.reduce(
        [float(alg_bytes), float(payload), float(cfg.streams)], "sum")
    e2e_max = coll.reduce([e2e_elapsed], "max")[0] if e2e_elapsed is not None else None
    if rank != 0:
        return None

    value = alg_total / t_max / 1e9
    exec_s = rep.exec_ms / 1e3
    exec_bytes = alg_bytes - eng["solve_bytes"]
    achieved = (exec_bytes / exec_s / 1e9) if exec_s > 0 else 0.0
    steps = args.steps
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
            "parallelism": "independent streams sharded by index (weak scaling)",
        },
        "payload_GBps": round(payload_total / t_max / 1e9, 3),
        "pct_hbm_peak": round(100.0 * value / (HBM_PEAK_GBPS * world), 2),
        "device": {
            "exec_ms_per_step": round(rep.exec_ms / steps, 3),
            "device_ms_per_step": round(rep.device_ms / steps, 3),
            "rounds_per_step": rep.rounds / steps,
            "launches_per_step": eng["launches"] / steps,
            "terms_per_step": eng["terms"] / steps,
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
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_exec",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": pmc_traffic("sgpu::k_exec"),
            "traffic_source": TRAFFIC_NOTE,
            "exec_bytes_per_step": exec_bytes // steps,
            "exec_launches_per_step": eng["exec_launches"] / steps,
            "exec_bytes_per_launch": exec_bytes // max(1, eng["exec_launches"]),
            "exec_ms_per_step": round(rep.exec_ms / steps, 4),
            "note": "achieved = k_exec's algorithmic bytes / summed k_exec launch time "
                    "(HIP events on the codec stream)",
        },
        "cpu_baseline": None,
        "end_to_end": None,
    }
    if e2e_max is not None:
        line["end_to_end"] = {
            "value": round(alg_total / e2e_max / 1e9, 3),
            "unit": "GB/s",
            "payload_GBps": round(payload_total / e2e_max / 1e9, 3),
            "ms_per_step": round(e2e_max / steps * 1e3, 3),
            "note": "originals H2D from pinned host memory each step; every recovery packet "
                    "and recovered original D2H (PCIe-inclusive; not `value`)",
        }
    if not args.no_cpu and world == 1:
        # the reference on the host cores, rank 0 at N=1 only
        threads = min(16, os.cpu_count() or 1)
        per_stream = alg_bytes / steps / args.streams
        line["cpu_baseline"] = cpu_baseline(args.cpu_streams, threads, per_stream)
    return line


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams", type=int, default=STREAMS_PER_GPU)
    ap.add_argument("--cpu-streams", type=int, default=16384)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--threads", type=int, default=0,
                    help="host threads driving streams (0 = library default)")
    ap.add_argument("--groups", type=int, default=2,
                    help="stream groups alternating host and device work (1 = no overlap)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false",
                    help="skip the PCIe-inclusive end-to-end leg")
    ap.add_argument("--library", default=S.AMD_LIB, help=argparse.SUPPRESS)
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = os.path.basename(args.library).startswith("libsiamese_amd")
    line = run_rank(rank, world, local, args, args.library, use_cuda)
    if line is not None:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
