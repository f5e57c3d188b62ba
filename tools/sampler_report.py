#!/usr/bin/env python3
"""Summarise tools/sampler.c output: self and inclusive sample counts per function.

usage: sampler_report.py PROF.txt [--filter SUBSTR] [--top N]
"""
import collections
import subprocess
import sys


def symbolize(frames):
    by_obj = collections.defaultdict(set)
    for fr in frames:
        obj, off = fr.rsplit(":", 1)
        by_obj[obj].add(off)
    names = {}
    for obj, offs in by_obj.items():
        offs = sorted(offs)
        if obj == "?":
            for o in offs:
                names["%s:%s" % (obj, o)] = "?"
            continue
        try:
            out = subprocess.run(["addr2line", "-f", "-C", "-e", obj] + ["0x" + o for o in offs],
                                 capture_output=True, text=True, check=True).stdout.splitlines()
        except (subprocess.CalledProcessError, OSError):
            out = ["?", "?"] * len(offs)
        for i, o in enumerate(offs):
            fn = out[2 * i] if 2 * i < len(out) else "?"
            if fn == "??":
                fn = "%s+%s" % (obj.rsplit("/", 1)[-1], o)
            names["%s:%s" % (obj, o)] = fn[:140]
    return names


def main():
    path = sys.argv[1]
    flt = None
    callers = None
    lines = False
    top = 40
    args = sys.argv[2:]
    while args:
        a = args.pop(0)
        if a == "--filter":
            flt = args.pop(0)
        elif a == "--lines":
            lines = True
        elif a == "--callers":
            callers = args.pop(0)
        elif a == "--top":
            top = int(args.pop(0))
    samples = []
    with open(path) as f:
        for line in f:
            parts = line.split()
            if parts and parts[0] == "S":
                samples.append(parts[1:])
    frames = {fr for s in samples for fr in s}
    names = symbolize(frames)
    if lines:
        # self samples of the filtered stacks by innermost source line
        # (inlined frames resolved), e.g. --filter sgpu_encoder_free --lines
        loc = collections.Counter()
        pcs = collections.defaultdict(list)
        for s in samples:
            syms = [names[fr] for fr in s]
            if flt and not any(flt in x for x in syms):
                continue
            if s:
                pcs[s[0]].append(1)
        by_obj = collections.defaultdict(list)
        for fr in pcs:
            obj, off = fr.rsplit(":", 1)
            by_obj[obj].append(off)
        for obj, offs in by_obj.items():
            out = subprocess.run(["addr2line", "-a", "-i", "-e", obj] + ["0x" + o for o in offs],
                                 capture_output=True, text=True).stdout.splitlines()
            cur = None
            for ln in out:
                if ln.startswith("0x"):
                    cur = obj + ":" + ("%x" % int(ln, 16))
                    first = True
                    continue
                if cur and first:
                    loc[ln.rsplit("/", 1)[-1]] += len(pcs.get(cur, []))
                    first = False
        for k, v in loc.most_common(top):
            print("%6d  %s" % (v, k))
        return
    if callers:
        chains = collections.Counter()
        for s in samples:
            syms = [names[fr] for fr in s]
            for i, x in enumerate(syms):
                if callers in x:
                    chains[" <- ".join(y[:60] for y in syms[i:i + 5])] += 1
                    break
        for k, v in chains.most_common(top):
            print("%6d  %s" % (v, k))
        return
    self_c = collections.Counter()
    incl_c = collections.Counter()
    total = 0
    for s in samples:
        syms = [names[fr] for fr in s]
        if flt and not any(flt in x for x in syms):
            continue
        total += 1
        if syms:
            self_c[syms[0]] += 1
        for x in set(syms):
            incl_c[x] += 1
    print("samples: %d" % total)
    print("--- self ---")
    for k, v in self_c.most_common(top):
        print("%6d %5.1f%%  %s" % (v, 100.0 * v / max(1, total), k))
    print("--- inclusive ---")
    for k, v in incl_c.most_common(top):
        print("%6d %5.1f%%  %s" % (v, 100.0 * v / max(1, total), k))


if __name__ == "__main__":
    main()
