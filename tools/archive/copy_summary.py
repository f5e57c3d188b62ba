"""Summarise a rocprofv3 memory-copy trace (csv): per direction, count, bytes,
summed duration and rate, plus the busy time of each stream's copies.
    python tools/copy_summary.py DIR"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
    if not f:
        print("no memory copy trace under", d)
        return
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(lambda: [0, 0, 0])
    for r in rows:
        k = r.get("Direction", "?")
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[k][0] += 1
        agg[k][1] += int(r.get("Bytes", 0) or 0)
        agg[k][2] += dur
    for k, (n, b, t) in sorted(agg.items()):
        print("%-24s n %6d  bytes %12d  time %9.3f ms  %7.1f GB/s" % (k, n, b, t / 1e6, b / max(t, 1)))
    big = sorted(rows, key=lambda r: -int(r.get("Bytes", 0) or 0))[:12]
    for r in big:
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print("  %-20s %10s B  %8.3f ms  %6.1f GB/s" % (r.get("Direction"), r.get("Bytes"), dur / 1e6,
                                                      int(r.get("Bytes", 0) or 0) / max(dur, 1)))


if __name__ == "__main__":
    main()
