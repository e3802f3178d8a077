#!/usr/bin/env python3
"""How much of each host<->device copy overlaps kernel execution, from a
rocprofv3 run with --kernel-trace --memory-copy-trace (host-resident input
bench, rten_hip/staging.py): the last N copies of the run, each with its
direction, duration, rate and the fraction of its interval during which some
kernel ran; then the kernel-busy fraction of the span they cover.
usage: copy_overlap.py <dir with run_kernel_trace.csv and run_memory_copy_trace.csv> [N]"""
import csv
import glob
import os
import sys


def load(d, name):
    f = glob.glob(os.path.join(d, "**", name), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in load(d, "run_kernel_trace.csv"))
    cs = load(d, "run_memory_copy_trace.csv")
    if not cs:
        print("no memory copy trace")
        return
    cs.sort(key=lambda r: int(r["Start_Timestamp"]))
    print("copy trace columns:", ",".join(cs[0].keys()), f"({len(cs)} copies)")

    def size_of(r):
        for k in ("Size", "Bytes", "Copy_Bytes", "Size_Bytes"):
            if r.get(k):
                return int(r[k])
        return 0

    big = [r for r in cs if size_of(r) >= 1 << 16 or (size_of(r) == 0 and
                                                       int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 50000)][-n:]

    def busy(a, b):
        t, cur = 0, a
        for s, e in ks:
            if e <= cur or s >= b:
                continue
            s2, e2 = max(s, cur), min(e, b)
            if e2 > s2:
                t += e2 - s2
                cur = e2
        return t

    for r in big:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        size = size_of(r)
        dirn = r.get("Direction", r.get("Operation", r.get("Kind", "?")))
        print(f"{dirn:>28} {size / 1e6:8.2f} MB {(b - a) / 1e3:8.1f} us {size / max(b - a, 1):6.1f} GB/s "
              f"kernel-overlap {busy(a, b) / max(b - a, 1):.2f}")
    if big:
        a = int(big[0]["Start_Timestamp"])
        b = max(int(r["End_Timestamp"]) for r in big)
        print(f"span {(b - a) / 1e3:.1f} us, kernels busy {busy(a, b) / max(b - a, 1):.3f} of it")


if __name__ == "__main__":
    main()
