#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Usage: pmc_traffic.py FETCH.csv WRITE.csv OUT.json [SOURCE-LABEL [LIBRARY.so [STEPS]]]

Both counters are reported in KiB per dispatch.  Following
MI355X_MICROARCH.md (HBM section), FETCH_SIZE on gfx950 counts half the
bytes of wide streaming reads and is doubled; WRITE_SIZE is taken as is.
Writes {kernel: {dispatches, fetch_bytes, write_bytes, traffic_bytes}}: the
byte figures are PER-DISPATCH AVERAGES (traffic_bytes_all is the sum over every
dispatch of the capture, traffic_bytes_max the largest dispatch).  With a
library path, "_lib_sha256" records the build the capture measured (bench.py
reports whether the library it loads is the same build).  STEPS: the workload
steps the captured process ran (bench.py runs --steps + --warmup + 2: the
verified warm-up and the unique-bytes step); "_step_traffic_bytes" is then
the traffic of all sgpu kernels per step (bench.py's physical step figure).
"""
import hashlib
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fb = 2.0 * sum(f) / len(f)
        wb = sum(w) / len(w)
        tot = [2.0 * a + b for a, b in zip(f, w)] if len(f) == len(w) else [fb + wb]
        out[k] = {"dispatches": len(f), "fetch_bytes": round(fb), "write_bytes": round(wb),
                  "traffic_bytes": round(fb + wb), "traffic_bytes_all": round(2.0 * sum(f) + sum(w)),
                  "traffic_bytes_max": round(max(tot))}
    out["_per"] = "dispatch (averages over the capture's dispatches)"
    if len(sys.argv) > 4:
        out["_source"] = sys.argv[4]
    if len(sys.argv) > 5:
        out["_lib_sha256"] = hashlib.sha256(open(sys.argv[5], "rb").read()).hexdigest()
    if len(sys.argv) > 6:
        steps = int(sys.argv[6])
        out["_workload_steps"] = steps
        out["_step_traffic_bytes"] = round(sum(v["traffic_bytes_all"] for k, v in out.items()
                                               if k.startswith("sgpu::")) / steps)
        out["_step_dispatches"] = {k: v["dispatches"] / steps for k, v in out.items() if k.startswith("sgpu::")}
    json.dump(out, open(sys.argv[3], "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
