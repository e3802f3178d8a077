#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (counter_collection.csv
files under a directory): kernel family (template arguments dropped) ->
counter -> mean value per dispatch, and the dispatch count.
usage: pmc_kernels.py DIR [name-filter]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"^void ", "", r["Kernel_Name"]).replace("(anonymous namespace)::", "")
            k = re.sub(r"\(.*$", "", k)
            if filt and filt not in k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, ctrs in sorted(acc.items()):
        n = max(len(v) for v in ctrs.values())
        print(f"{k}  ({n} dispatches)")
        for c, v in sorted(ctrs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
