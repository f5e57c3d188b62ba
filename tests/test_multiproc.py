"""The N>1 bench path on CPU: two gloo ranks, each running its own shard of
streams through the control plane (CPU test double of the backend), with the
barrier / max-time / sum reductions of bench.py.  The union of the two
shards must equal one process running all the streams."""
import json
import os
import subprocess
import sys

import scenario_lib as S

ROOT = S.ROOT


BENCH_ARGS = ["--library", S.SIM_LIB, "--streams", "6", "--steps", "1", "--warmup", "1",
              "--no-cpu", "--no-legs"]


def _clean_env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_gpus_2_spawns_two_ranks():
    """`bench.py --gpus 2` with no WORLD_SIZE starts its own two rank
    processes (the driver's SCALE run) and reports the 2-rank aggregate."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] +
                       BENCH_ARGS, env=_clean_env(), capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout   # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["streams_total"] == 12
    assert "gloo" in line["config"]["parallelism"]


def test_two_rank_gloo_bench_shards_streams():
    env = dict(_clean_env(), MASTER_ADDR="127.0.0.1", MASTER_PORT="29517")
    procs = []
    for rank in range(2):
        e = dict(env, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "bench.py")] + BENCH_ARGS,
            env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=600) for p in procs]
    for p, (o, err) in zip(procs, outs):
        assert p.returncode == 0, err[-2000:]
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    # only rank 0 prints the JSON line (gloo itself may log to stdout)
    assert not any(l.startswith("{") for l in outs[1][0].splitlines())
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["streams_total"] == 12

    # union of the shards == one run over streams 0..11 (same digests)
    whole = S.replace(S.CONFIGS["C4"], streams=12, hash_data=0)
    ref, _ = S.run_batch(S.SIM_LIB, whole, verify=False)
    shard0 = S.replace(whole, streams=6, first_stream=0)
    res0, _ = S.run_batch(S.SIM_LIB, shard0, verify=False)
    shard1 = S.replace(whole, streams=6, first_stream=6)
    res1, _ = S.run_batch(S.SIM_LIB, shard1, verify=False)
    assert S.digests(res0) + S.digests(res1) == S.digests(ref)
