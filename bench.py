#!/usr/bin/env python3
"""bench.py -- device-resident encode+decode throughput of the MI355X
streaming erasure codec (BASELINE.json metric), one JSON line on rank 0.

Workload (per GPU, weak scaling): the C4 shard -- 1024 independent streams x
256 originals x 1400 B, 20% loss on originals and recovery packets, block
mode (all originals added, then recovery packets until every original is
delivered).  8 GPUs x 1024 streams = C4's 8192 streams; rank r runs global
streams [1024 r, 1024 (r+1)), so no data-path collective exists.

A "step" is that whole workload: create 1024 encoder/decoder pairs, ingest
the originals (already resident in HBM), encode, drop, decode, verify the
control flow, free.  Timing covers the full step: host control plane and
device work.

value  = algorithmic bytes / step time, summed over ranks (GB/s), where the
         algorithmic bytes are the source bytes of every GF(256)
         add/mul/muladd the reference codec performs for the same call
         sequence plus the recovery packets and recovered originals written
         (counted by the library, cross-checked against the
         instrumented reference in tests/).
roofline = the executor kernel (k_exec): its share of the algorithmic bytes
         over its measured device time (HIP events on the codec's stream),
         against the 8 TB/s HBM3E peak.
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
        "sample": "%d C4 streams (256 x 1400 B, 20%% loss, block) on %d threads, %.2f s"
                  % (sample_streams, threads, wall),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--streams", type=int, default=STREAMS_PER_GPU)
    ap.add_argument("--cpu-streams", type=int, default=4096)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    cfg = workload(rank, args.streams)
    sess = S.BatchSession(S.AMD_LIB, cfg, device=local)
    # verified, untimed run first: every recovered byte is compared with its payload
    res, rep = sess.run(steps=0, warmup=max(1, args.warmup), verify=True)
    if rep.mismatches or any(r.status for r in res):
        print("bench: verification failed: %d mismatches, status %s" %
              (rep.mismatches, S.summary(res)["status"]), file=sys.stderr)
        sys.exit(1)

    barrier()
    t0 = time.perf_counter()
    res, rep = sess.run(steps=args.steps, warmup=0, verify=False)
    barrier()
    elapsed = time.perf_counter() - t0
    sess.close()

    eng = S.engine_dict(rep)
    alg_bytes = eng["ref_op_bytes"] + eng["out_bytes"]        # over all timed steps
    payload = sum(r.payload_bytes for r in res) * args.steps
    stats = torch.tensor([elapsed, rep.exec_ms, rep.device_ms, float(alg_bytes),
                          float(payload)], dtype=torch.float64, device="cuda")
    if dist is not None:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        t_max, alg_total, payload_total = float(mx[0]), float(sm[3]), float(sm[4])
    else:
        t_max, alg_total, payload_total = elapsed, float(alg_bytes), float(payload)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    value = alg_total / t_max / 1e9
    # Roofline of the dominant kernel k_exec: its share of the algorithmic
    # bytes (everything except the triangular solve, which runs in the
    # k_solve_* kernels) over its own summed launch time.
    exec_s = rep.exec_ms / 1e3
    exec_bytes = alg_bytes - eng["solve_bytes"]
    achieved = (exec_bytes / exec_s / 1e9) if exec_s > 0 else 0.0
    launches = max(1, eng["launches"])
    line = {
        "metric": "device-resident GB/s encode+decode, 1400B pkts @20% loss; % HBM peak",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (reference unit_test SetPacket payloads, PCG loss channel seed 1013)",
        "config": {
            "workload": "C4 shard per GPU: %d streams x 256 originals x 1400 B, 20%% loss, "
                        "block mode, no RCCL" % args.streams,
            "streams_per_gpu": args.streams,
            "streams_total": args.streams * world,
            "originals": 256,
            "payload_bytes": 1400,
            "loss_pct": 20,
            "parallelism": "independent streams sharded by index (weak scaling)",
        },
        "payload_GBps": round(payload_total / t_max / 1e9, 3),
        "pct_hbm_peak": round(100.0 * value / (HBM_PEAK_GBPS * world), 2),
        "device": {
            "exec_ms_per_step": round(rep.exec_ms / args.steps, 3),
            "device_ms_per_step": round(rep.device_ms / args.steps, 3),
            "rounds_per_step": rep.rounds / args.steps,
            "launches_per_step": eng["launches"] / args.steps,
            "terms_per_step": eng["terms"] / args.steps,
            "algorithmic_bytes_per_step": alg_bytes // args.steps,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_exec",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": None,
            "exec_bytes_per_step": exec_bytes // args.steps,
            "exec_ms_per_step": round(rep.exec_ms / args.steps, 4),
            "note": "achieved = k_exec's algorithmic bytes / summed k_exec launch time "
                    "(HIP events on the codec stream); %d launches/step of all kernels"
                    % (launches // args.steps),
        },
        "cpu_baseline": None,
    }
    if not args.no_cpu:
        threads = min(16, os.cpu_count() or 1)
        per_stream = alg_bytes / args.steps / args.streams
        line["cpu_baseline"] = cpu_baseline(args.cpu_streams, threads, per_stream)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
