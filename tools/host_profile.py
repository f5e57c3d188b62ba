#!/usr/bin/env python3
"""Run bench.py under the SIGPROF sampler (tools/sampler.c) loaded in-process.

usage: python tools/host_profile.py OUT_PREFIX [bench.py args...]
writes OUT_PREFIX.<pid>; summarise with tools/sampler_report.py.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    os.environ["SAMPLER_OUT"] = sys.argv[1]
    # bring the GPU runtime up before any sampling signal can interrupt its
    # initialisation (an interrupted device probe reads as "no GPU")
    import torch
    if torch.cuda.is_available():
        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    ctypes.CDLL(os.path.join(ROOT, "tools", "libsampler.so"))   # constructor starts the timer
    sys.path.insert(0, ROOT)
    import bench
    bench.main(sys.argv[2:])
