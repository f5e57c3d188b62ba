#!/usr/bin/env python3
"""Build a patched copy of the product library for A/B timing on the GPU box:
  python tools/variant_src.py NAME SPEC.py [-DFOO ...]
SPEC.py defines PATCHES = [(file, old, new), ...]: exact replacements applied
to a copy of siamese_amd/csrc (each `old` must occur).  Produces
siamese_amd/libsiamese_amd_NAME.so (git-ignored); the product sources are
not touched.  Timing variants may compute wrong outputs: run them with
`bench.py --no-verify --library ...`."""
import os
import runpy
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, spec = sys.argv[1], sys.argv[2]
defs = sys.argv[3:]
src = os.path.join(ROOT, "siamese_amd", "csrc")
dst = os.path.join(ROOT, "vbuild", name)   # (two levels down: the sources include ../../include)
shutil.rmtree(dst, ignore_errors=True)
shutil.copytree(src, dst)
specd = runpy.run_path(spec)
for f, old, new in specd.get("PATCHES", []):
    p = os.path.join(dst, f)
    s = open(p).read()
    if old not in s:
        sys.exit("patch not found in %s: %r" % (f, old[:80]))
    open(p, "w").write(s.replace(old, new, 1))
if "transform" in specd:
    # transform(name, text) -> text, for every copied source file
    for f in sorted(os.listdir(dst)):
        p = os.path.join(dst, f)
        if os.path.isfile(p):
            s = open(p).read()
            t = specd["transform"](f, s)
            if t != s:
                open(p, "w").write(t)
obj = os.path.join(dst, "obj")
os.makedirs(obj)
procs = []
for f in "gf codedef pool placement engine encoder decoder arq api batch frames".split():
    procs.append(subprocess.Popen(["g++", "-std=c++17", "-O2", "-g", "-mavx2", "-fPIC", "-ftls-model=initial-exec",
                                   "-fvisibility=hidden"] + defs + ["-c", os.path.join(dst, f + ".cpp"), "-o",
                                   os.path.join(obj, f + ".o")]))
subprocess.check_call(["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", "-fPIC",
                       "-ftls-model=initial-exec", "-fvisibility=hidden", "-Wno-unused-parameter",
                       "-Wno-unused-result"] + defs + ["-c", os.path.join(dst, "backend_hip.hip"), "-o",
                       os.path.join(obj, "backend_hip.o")])
for p in procs:
    if p.wait():
        sys.exit("host compile failed")
out = os.path.join(ROOT, "siamese_amd", "libsiamese_amd_%s.so" % name)
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] +
                      [os.path.join(obj, f) for f in sorted(os.listdir(obj))] + ["-lpthread"])
print("built", os.path.relpath(out, ROOT))
