#!/usr/bin/env python3
"""Summary of l2_hot_cold.py's rocprofv3 kernel trace: median duration of
the conv kernel the replays run (the cold phase's most frequent kernel)
before (hot) and after (cold) the first fill kernel (the marker).
usage: l2_hot_cold_summary.py run_kernel_trace.csv"""
import collections
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
cut = next((i for i, r in enumerate(rows) if "at::native" in r["Kernel_Name"]), len(rows) // 2)
names = collections.Counter(r["Kernel_Name"] for r in rows[cut:] if "gemm_" in r["Kernel_Name"] or "conv_" in r["Kernel_Name"])
name = names.most_common(1)[0][0]
hot = [dur(r) for r in rows[:cut] if r["Kernel_Name"] == name][-40:]
cold = [dur(r) for r in rows[cut:] if r["Kernel_Name"] == name][-40:]
print(f"{name[:70]}: hot median {statistics.median(hot):.2f} us ({len(hot)}), "
      f"cold median {statistics.median(cold):.2f} us ({len(cold)})")
