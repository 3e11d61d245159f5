#!/usr/bin/env python
"""Average duration per kernel (us) from rocprofv3 kernel_stats.csv files: kstats.py [--match SUBSTR] FILE..."""
import csv
import sys

args = sys.argv[1:]
match = ""
if args[:1] == ["--match"]:
    match, args = args[1], args[2:]
for f in args:
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows:
        if match in r["Name"]:
            print("%-40s %9.1f us x %4s  %s" % (f[-40:], float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:60]))
