#!/usr/bin/env python3
"""Per-forward kernel summary from a rocprofv3 kernel trace (run_kernel_trace.csv).

rocprofv3's --stats averages every dispatch of the run, including the
plan-time tuner's candidate launches; this keeps only the steady state: the
trailing dispatches, cut into forwards by the period of the kernel-name
sequence, and reports per kernel (template arguments dropped) the time and
launches per forward and the average launch duration.
usage: rocprof_per_forward.py run_kernel_trace.csv [forwards] [min_period] [--seq]
(ROCclr fill / copy kernels are counted like any other dispatch.)
(--seq: also list one forward's dispatches in order, each with its duration
and the gap since the previous dispatch ended, averaged over the forwards)
(min_period: dispatches per forward at least -- BERT's layers repeat inside a
forward, so its period is given as more than 12 layers x 7 dispatches, e.g. 85)"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return re.sub(r"[<(].*$", "", name)


def main():
    seq = "--seq" in sys.argv
    argv = [a for a in sys.argv if a != "--seq"]
    path = argv[1]
    want = int(argv[2]) if len(argv) > 2 else 10
    min_period = int(argv[3]) if len(argv) > 3 else 4
    # ROCclr's own fill / copy kernels (hipMemsetAsync / hipMemcpyAsync inside
    # the step) are kept: they are part of the forward and explain gaps.
    rows = list(csv.DictReader(open(path)))
    # (bench.py's per-op timing runs hold the stream with rtenhip::hold_kernel
    # until their plan is queued: a timing artefact, not part of a forward.)
    # They follow the timed replays and run eagerly with an event around every
    # op (each event a cache flush, so their kernels run slower): the steady
    # state is the stretch before the first of them.
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first_hold = next((i for i, r in enumerate(rows) if "hold_kernel" in r["Kernel_Name"]), None)
    if first_hold is not None:
        rows = rows[:first_hold]
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
    if seq:
        print("--- one forward, in dispatch order (us, averaged over the forwards) ---")
        for i in range(period):
            durs, gaps = [], []
            for f in range(n):
                r = tail[f * period + i]
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                if f * period + i > 0:
                    prev = tail[f * period + i - 1]
                    gaps.append(int(r["Start_Timestamp"]) - int(prev["End_Timestamp"]))
            name = re.sub(r"^void (rtenhip::)?", "", tail[i]["Kernel_Name"].replace("(anonymous namespace)::", ""))
            name = re.sub(r"\(.*$", "", name)
            g = sum(gaps) / len(gaps) / 1e3 if gaps else 0.0
            print(f"  {i:3d} {sum(durs) / len(durs) / 1e3:8.2f} gap {g:6.2f}  {name[:90]}")


if __name__ == "__main__":
    main()
