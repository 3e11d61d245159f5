#!/usr/bin/env python
"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh output): per kernel, the mean
per-dispatch value of every counter collected.   python scripts/pmc_summary.py gpurun_out/pmc"""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per-dispatch values]
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)   # (kernel, dispatch, counter) -> summed over dimensions
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "")
            per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


if __name__ == "__main__":
    s = summarise(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
    for k in sorted(s):
        print(k)
        for c in sorted(s[k]):
            print("    %-28s %16.1f" % (c, s[k][c]))
