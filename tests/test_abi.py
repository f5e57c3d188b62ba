"""The C-ABI boundary: every entry point declared in include/*.h is exported by
the product library (and by the CPU test double), the library loads without a
GPU and refuses to run without one (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

import scenario_lib as S

HEADERS = [os.path.join(S.ROOT, "include", h) for h in ("siamese.h", "siamese_gpu.h")]


def declared(header):
    text = open(header).read()
    return sorted(set(re.findall(r"SIAMESE_EXPORT\s+[\w\s\*]+?\b(\w+)\s*\(", text)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_headers_declare_the_reference_api():
    names = declared(HEADERS[0])
    assert len(names) == 20
    assert "siamese_encode" in names and "siamese_decode" in names and "siamese_init_" in names


@pytest.mark.parametrize("lib", [S.AMD_LIB, S.SIM_LIB])
def test_library_exports_every_declared_symbol(lib):
    have = exported(lib)
    for h in HEADERS:
        missing = [n for n in declared(h) if n not in have]
        assert not missing, "%s misses %s from %s" % (lib, missing, h)


def test_reference_exports_match_our_siamese_h():
    if not os.path.exists(S.REF_LIB):
        pytest.skip("oracle/_ref not built")
    ref = {n for n in exported(S.REF_LIB) if n.startswith("siamese_")}
    assert ref == set(declared(HEADERS[0]))


def test_product_library_has_no_cpu_backend():
    """The shipped library links the HIP backend only: the test double's
    symbols must not be in it."""
    out = subprocess.run(["nm", "-C", S.AMD_LIB], capture_output=True, text=True).stdout
    assert "hostsim" not in out
    assert "k_exec" in out  # the gfx950 executor kernel stub


def test_product_refuses_to_run_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    L = ctypes.CDLL(S.AMD_LIB)
    assert L.siamese_init_(5) == 5  # Siamese_Disabled: loud failure, no fallback
    L.siamese_encoder_create.restype = ctypes.c_void_p
    assert not L.siamese_encoder_create()
