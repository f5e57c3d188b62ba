"""CPU parity of the host control plane.

* The reference build (oracle/_ref) reproduces the committed golden digests,
  so the fixtures and the harness are pinned.
* The control plane of libsiamese_amd, linked against the CPU test double of
  its backend (tests/hostsim -- never shipped), reproduces the reference
  digests through both the drop-in per-call API and the batched device API.
The same comparisons run on the MI355X with the real HIP backend in
test_gpu_parity.py.
"""
import os

import pytest

import golden
import scenario_lib as S

SMALL = ["smoke_C4x8", "C1", "C1var", "C2x64", "edge_tiny", "edge_var_block", "edge_heavy",
         "edge_maxloss", "edge_lag", "smoke_C4x8r", "edge_var_block_r", "C2x64r", "C1r", "C1var_r"]


def _check(name, results):
    want = golden.load(name)
    got = S.digests(results)
    bad = [i for i, (a, b) in enumerate(zip(got, want["digests"])) if a != b]
    assert not bad, "%s: %d/%d streams differ (first %s)" % (name, len(bad), len(got), bad[:5])
    assert [int(r.status) for r in results] == want["status"]


@pytest.mark.parametrize("name", SMALL + ["C3", "C4x256", "C2", "C2h", "C2hr", "C4x1024h", "C4x1024hr"])
def test_reference_matches_golden(name, ref_available):
    if not ref_available:
        pytest.skip("oracle/_ref not built")
    cfg = golden.config(name)
    res, _, _ = S.run_capi(S.REF_LIB, cfg, threads=min(8, cfg.streams))
    _check(name, res)


@pytest.mark.parametrize("name", SMALL)
def test_hostsim_dropin_matches_golden(name):
    cfg = golden.config(name)
    res, _, _ = S.run_capi(S.SIM_LIB, cfg)
    _check(name, res)


@pytest.mark.parametrize("name", ["C2x64", "smoke_C4x8", "C1var"])
def test_hostsim_dropin_threads_match_golden(name):
    """siamese.h from several threads at once, each driving its own streams:
    instance calls run concurrently under the shared instance lock and their
    flushes commit as groups; every stream's digest is the reference's."""
    cfg = golden.config(name)
    res, _, _ = S.run_capi(S.SIM_LIB, cfg, threads=min(8, cfg.streams))
    _check(name, res)


@pytest.mark.parametrize("name", SMALL)
def test_hostsim_batch_matches_golden(name):
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True)
    _check(name, res)
    assert rep.mismatches == 0


@pytest.mark.parametrize("name", ["C2x64", "C1var", "edge_lag", "smoke_C4x8", "edge_var_block_r"])
@pytest.mark.parametrize("threads,groups", [(1, 2), (4, 2), (8, 3)])
def test_hostsim_batch_threads_and_pipelining(name, threads, groups):
    """Streams driven from several host threads (per-thread engine shards)
    and split into groups whose flushes overlap the other groups' host work
    give the reference's results."""
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, threads=threads, groups=groups)
    _check(name, res)
    assert rep.mismatches == 0


def test_hostsim_batch_length_only_digest():
    """hash_data=0 digests (used for the full-size GPU runs) also agree."""
    cfg = S.replace(golden.config("C4x256"), streams=32, hash_data=0)
    ref, _, _ = S.run_capi(S.REF_LIB, cfg, threads=8) if os.path.exists(S.REF_LIB) else (None,) * 3
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True)
    assert rep.mismatches == 0 and rep.checked > 0
    if ref is not None:
        assert S.digests(res) == S.digests(ref)


@pytest.mark.parametrize("name", ["C2x64", "smoke_C4x8"])
def test_hostsim_batch_end_to_end_pipelined(name):
    """End-to-end mode: the originals arrive by asynchronous copies into two
    device copies that alternate by step (sgpu_h2d_async), results come back
    through the gather stream into pinned memory (sgpu_gather_completed);
    several pipelined steps verify every recovered byte."""
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, steps=3, verify=True, threads=4, groups=2, e2e=True)
    _check(name, res)
    assert rep.mismatches == 0 and rep.checked > 0


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("defer", [1, 3])
def test_hostsim_deferred_outputs_match_golden(name, defer):
    """Deferred outputs (sgpu_decode_deferred / sgpu_decoder_get_deferred): a
    stream yields only after every `defer`-th decode and each group keeps two
    submissions in flight, so instances are driven while their solves are
    still pending (recovered lengths are bounds until the completion is
    applied).  Every byte is verified and the digests are the reference's."""
    cfg = golden.config(name)
    res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, defer=defer, threads=4,
                           groups=2 if cfg.streams >= 8 else 1)
    _check(name, res)
    assert rep.mismatches == 0


@pytest.mark.parametrize("name", ["edge_lag", "C1var", "edge_var_block"])
def test_hostsim_deferred_length_only(name):
    """Length-only digests (hash_data=0: no yield after each encode) with
    variable packet sizes: the rounds hold several decodes with recovered
    lengths still pending, and every recovered byte must still verify."""
    cfg = S.replace(golden.config(name), hash_data=0)
    ref, _, _ = S.run_capi(S.REF_LIB, cfg) if os.path.exists(S.REF_LIB) else (None, 0, 0)
    for defer in (1, 4):
        res, rep = S.run_batch(S.SIM_LIB, cfg, verify=True, defer=defer, threads=4)
        assert rep.mismatches == 0 and rep.checked > 0
        assert not any(r.status for r in res)
        if ref is not None:
            assert S.digests(res) == S.digests(ref)
