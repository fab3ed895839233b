#!/usr/bin/env python
"""Per-kernel (full template name) per-dispatch averages of every counter in rocprofv3 --pmc CSVs under a
directory (one or more passes).  Usage: python tools/pmc_kernels.py DIR [name-filter]"""
import collections
import csv
import glob
import os
import sys


def main(root, filt=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if filt not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    for k, v in sorted(agg.items()):
        print(k)
        for c in sorted(v):
            print(f"    {c:28s} {v[c] / max(len(disp[k][c]), 1):16.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
