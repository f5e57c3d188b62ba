"""Symbolize tools/malloc_sites.c output: python tools/malloc_report.py FILE [N] [--map FROM=TO]"""
import subprocess
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 30
maps = [a.split("=", 1) for a in sys.argv[2:] if "=" in a]
lines = open(path).read().splitlines()
print(lines[0])
cache = {}


def sym(fr):
    if fr in cache:
        return cache[fr]
    obj, off = fr.rsplit("+", 1)
    for a, b in maps:
        obj = obj.replace(a, b)
    try:
        out = subprocess.run(["addr2line", "-f", "-C", "-e", obj, "0x" + off], capture_output=True,
                             text=True).stdout.splitlines()
        name = out[0][:60] if out and out[0] != "??" else obj.rsplit("/", 1)[-1] + "+" + off
    except OSError:
        name = fr
    cache[fr] = name
    return name


for l in lines[1:top + 1]:
    p = l.split()
    print(p[0], " <- ".join(sym(x) for x in p[1:6] if "+" in x))
