"""The algorithmic bytes behind bench.py's `value`:
the source bytes of every bulk GF(256) op the reference codec performs for
the same call sequence.

oracle/_ref/libsiamese_ref_counted.so is the unmodified reference with every
call into gf256_{add,mul,muladd}_mem counted (oracle/opcount.c, linker
--wrap).  Our library counts the same quantity while it runs: on the host for
the ops it emits, on the device for the terms the executor expands itself
(lane-sum updates, LDPC picks).  The two must agree byte for byte.

Known deviation: on streaming runs that mix variable packet lengths with
acknowledgements (C1var, edge_lag) the decoder folds some recovered originals
into its running sums through GetSum where the reference plugs them in
through PlugSumHoles (the same XOR, a different op trace), so the counts
differ by under 0.5 %; recovered bytes are identical (the digests match).
"""
import ctypes
import os

import pytest

import golden
import scenario_lib as S

COUNTED = os.path.join(S.ROOT, "oracle", "_ref", "libsiamese_ref_counted.so")

EXACT = ["C1", "C2x64", "edge_tiny", "edge_var_block", "edge_heavy", "edge_maxloss", "smoke_C4x8"]
NEAR = ["C1var", "edge_lag"]


def reference_op_bytes(cfg):
    lib = ctypes.CDLL(COUNTED)
    lib.ref_op_bytes.restype = ctypes.c_uint64
    lib.ref_op_bytes.argtypes = [ctypes.c_int]
    lib.ref_op_bytes(1)
    res, _, _ = S.run_capi(COUNTED, cfg)
    return lib.ref_op_bytes(1), res


def ours(library, cfg):
    res, rep = S.run_batch(library, cfg, verify=False)
    return S.engine_dict(rep)["ref_op_bytes"], res


def _need_counted():
    if not os.path.exists(COUNTED):
        pytest.skip("oracle/_ref/libsiamese_ref_counted.so not built")


@pytest.mark.parametrize("name", EXACT + ["C3x1500"])
def test_hostsim_op_bytes_equal_reference(name):
    _need_counted()
    cfg = (S.replace(S.CONFIGS["C3"], originals=1500) if name == "C3x1500" else golden.config(name))
    want, ref = reference_op_bytes(cfg)
    got, res = ours(S.SIM_LIB, cfg)
    assert S.digests(res) == S.digests(ref)
    assert got == want


@pytest.mark.parametrize("name", NEAR)
def test_hostsim_op_bytes_near_reference(name):
    _need_counted()
    cfg = golden.config(name)
    want, ref = reference_op_bytes(cfg)
    got, res = ours(S.SIM_LIB, cfg)
    assert S.digests(res) == S.digests(ref)
    assert abs(got - want) <= 0.005 * want


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["smoke_C4x8", "C2x64", "C1"])
def test_device_op_bytes_equal_reference(name):
    """On the MI355X the executor counts its expanded terms with atomics."""
    _need_counted()
    cfg = golden.config(name)
    want, _ = reference_op_bytes(cfg)
    got, _ = ours(S.AMD_LIB, cfg)
    assert got == want
