#!/usr/bin/env python3
"""Per-forward kernel summary from a rocprofv3 kernel trace (run_kernel_trace.csv).

rocprofv3's --stats averages every dispatch of the run, including the
plan-time tuner's candidate launches; this keeps only the steady state: the
trailing dispatches, cut into forwards by the period of the kernel-name
sequence, and reports per kernel (template arguments dropped) the time and
launches per forward and the average launch duration.
usage: rocprof_per_forward.py run_kernel_trace.csv [forwards] [min_period]
(min_period: dispatches per forward at least -- BERT's layers repeat inside a
forward, so its period is given as 12 layers x 13 dispatches = 156)"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    return re.sub(r"[<(].*$", "", name)


def main():
    path = sys.argv[1]
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    min_period = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    rows = [r for r in csv.DictReader(open(path)) if "rocclr" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # smallest period p of the trailing sequence that repeats at least twice
    period = None
    for p in range(min_period, len(names) // 2 + 1):
        if names[-p:] == names[-2 * p:-p]:
            period = p
            break
    if period is None:
        sys.exit("no repeating forward found")
    n = 1
    while n < want and len(names) >= (n + 1) * period and names[-(n + 1) * period:-n * period] == names[-period:]:
        n += 1
    tail = rows[-n * period:]
    t0 = int(tail[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in tail)
    # union of kernel intervals (side streams overlap)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tail)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    per = defaultdict(lambda: [0, 0])
    for r in tail:
        k = short(r["Kernel_Name"])
        per[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[k][1] += 1
    print(f"{n} forwards: {len(tail)} dispatches, wall span {(t1 - t0) / 1e6:.3f} ms "
          f"({(t1 - t0) / 1e6 / n:.4f} ms/forward), GPU busy (union of kernels) {busy / 1e6 / n:.4f} ms/forward")
    for k, (ns, c) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:42s} {ns / 1e6 / n:8.4f} ms/forward {c // n:5d} launches/forward  avg {ns / c / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
