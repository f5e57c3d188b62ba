"""Recovery matrix on the device (sgpu_decode_device, kernel k_ge): CPU
parity through the backend's CPU test double (tests/hostsim, never shipped).

A decode that starts a fresh elimination queues the matrix job and returns
SGPU_DECODE_PENDING; the call after the flush finishes it.  The harness logs
one EV_DECODE per decode, so the event digests must be the reference's
exactly, and the algorithmic bytes (the elimination's multiplies are counted
by the job) those of the host elimination.  The same checks run on the
MI355X in test_gpu_parity.py.
"""
import pytest

import golden
import scenario_lib as S
from test_parity_cpu import SMALL, _check


@pytest.mark.parametrize("name", SMALL + ["C2x64"])
def test_device_ge_matches_golden(name):
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, device_ge=True)
    _check(name, res)
    assert rep.mismatches == 0


@pytest.mark.parametrize("name", ["C2x64", "C1var", "smoke_C4x8", "edge_maxloss", "edge_heavy"])
@pytest.mark.parametrize("threads,groups", [(4, 2), (8, 3)])
def test_device_ge_threads_and_pipelining(name, threads, groups):
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, threads=threads, groups=groups, device_ge=True)
    _check(name, res)
    assert rep.mismatches == 0


@pytest.mark.parametrize("name,jobs", [("smoke_C4x8", True), ("C2x64", True), ("C1var", True),
                                       ("edge_lag", True), ("edge_maxloss", True)])
def test_device_ge_accounting_and_launches(name, jobs):
    """Same algorithmic bytes as the host elimination; the jobs ran (one more
    launch per flush that carried any).  edge_maxloss's decodes of more than
    128 lost columns run on the device too (k_ge takes the reference's 255)."""
    cfg = golden.config(name)
    _, rep0 = S.run_batch(S.SIM_LIB, cfg, verify=True)
    _, rep1 = S.run_batch(S.SIM_LIB, cfg, verify=True, device_ge=True)
    e0, e1 = S.engine_dict(rep0), S.engine_dict(rep1)
    assert e1["ref_op_bytes"] == e0["ref_op_bytes"]
    assert e1["out_bytes"] == e0["out_bytes"]
    assert (e1["launches"] > e0["launches"]) == jobs


def test_device_ge_headline_shard_slice():
    """A slice of the bench workload (C4 block mode, hashed) in range mode."""
    cfg = S.replace(golden.config("C4x1024hr"), streams=96)
    ref = golden.load("C4x1024hr")
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, threads=4, groups=2, device_ge=True)
    assert S.digests(res) == ref["digests"][:96]
    assert rep.mismatches == 0


@pytest.mark.parametrize("name,streams", [("C4x1024hr", 256), ("edge_lag", None), ("C2x64", None)])
def test_chained_decodes_and_singular_retries(name, streams):
    """Chained device decodes (DecoderCore::submit_chained): the matrix job,
    the elimination of received data and the solve in one submission, the
    last two gated on the job's outcome.  These fixtures hold first attempts
    whose square matrix is singular (the gated work must not run, the sums go
    back to their state before it, and the host repeats the elimination as
    the reference does): digests and algorithmic bytes stay the host path's."""
    cfg = golden.config(name)
    if streams:
        cfg = S.replace(cfg, streams=streams)
    want = golden.load(name)["digests"]
    res0, rep0 = S.run_batch(S.SIM_LIB, cfg, verify=True, threads=4, groups=2)
    res1, rep1 = S.run_batch(S.SIM_LIB, cfg, verify=True, threads=4, groups=2, device_ge=True)
    e0, e1 = S.engine_dict(rep0), S.engine_dict(rep1)
    assert S.digests(res1) == want[:len(S.digests(res1))]
    assert rep1.mismatches == 0
    assert e1["ref_op_bytes"] == e0["ref_op_bytes"]
    assert e1["out_bytes"] == e0["out_bytes"]
    assert e1["ge_chained"] > 0
    if name != "C2x64":
        assert e1["ge_retried"] >= 1   # (a singular first attempt is in these fixtures)
    if name == "C4x1024hr":
        assert e1["ge_chained"] == e1["ge_jobs"]   # (block decodes: every one chained)
