"""Print name, calls, average and max ns of each kernel in a rocprofv3 --stats directory.
usage: python3 tools/kstats.py DIR"""
import csv
import glob
import sys

for f in glob.glob(sys.argv[1] + "/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print("%-28s %5s %12.0f %10s" % (r["Name"].split("(")[0], r["Calls"], float(r["AverageNs"]), r["MaxNs"]))
