#!/usr/bin/env python3
"""Per-call-kind timing of C1 through the drop-in siamese.h ABI
(SCENARIO_CAPI_CALLS): python tools/dropin_probe.py [library] [runs]"""
import os
import sys

os.environ["SCENARIO_CAPI_CALLS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenario_lib as S  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else S.AMD_LIB
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = S.CONFIGS["C1"]
for i in range(runs):
    res, sec = S.run_capi(lib, cfg)[:2]
    print("run %d: %.3f ms codec" % (i, sec * 1e3), flush=True)
