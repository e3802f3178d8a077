#!/usr/bin/env python3
"""Durations of the last N dispatches of a rocprofv3 kernel trace whose
names match a pattern (default: the latency GEMM kernels), in order.
usage: last_forward.py run_kernel_trace.csv N [pattern]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rocclr" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
pat = sys.argv[3] if len(sys.argv) > 3 else "gemm_lat"
tail = rows[-n:]
i = 0
for r in tail:
    if pat in r["Kernel_Name"]:
        i += 1
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        print(f"{i:3d} {d:8.2f} us  {r['Kernel_Name'][:70]}")
