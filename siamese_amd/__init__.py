"""siamese_amd -- MI355X-native streaming erasure codec (Siamese-compatible).

The codec itself is native: libsiamese_amd.so (C++ control plane + gfx950 HIP
kernels) exporting the upstream siamese.h C ABI plus the device-resident batch
API of include/siamese_gpu.h.  This module is a thin ctypes binding used by
the tests and the benchmark; it has no compute path of its own and raises if
the native library or the GPU is missing.
"""
import os

from .binding import (SiameseLib, SiameseError, Success, InvalidInput, NeedMoreData,  # noqa: F401
                      MaxPacketsReached, DuplicateData, Disabled, RESULT_NAMES)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsiamese_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError("siamese_amd: %s is missing -- run __graft_entry__.build() "
                      "(there is no CPU fallback)" % LIB_PATH)

lib = SiameseLib(LIB_PATH)


def require_gpu():
    """siamese_init() on the device library; raises if no MI355X is usable."""
    lib.init()
    return lib


def Encoder():
    return lib.Encoder()


def Decoder():
    return lib.Decoder()
