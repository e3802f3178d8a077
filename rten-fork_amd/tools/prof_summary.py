#!/usr/bin/env python3
"""Per-step kernel time of the bench's timed region from a rocprofv3
--kernel-trace CSV: the last STEPS forwards (each = 53 gemm_dma_kernel
dispatches + the other ops) are located by walking back from the end of the
trace past the eager timing-report runs.  Prints per-kernel-family totals per
forward so they can be set beside bench.py's roofline.kernel_ms_per_step.

usage: prof_summary.py run_kernel_trace.csv [forwards=10] [skip_last_forwards=0]
(skip_last_forwards: e.g. bench's eager timing-report runs after the timed
hipGraph steps)."""
import csv
import sys
from collections import defaultdict


def family(name):
    n = name.split("(")[0].replace("void ", "")
    return n.split("<")[0]


def main():
    path = sys.argv[1]
    fwd = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # A forward = the span from one stem conv (first gemm_dma after the
    # previous forward's FC gemm) ... take the last `fwd` forwards by counting
    # gemm_dma dispatches from the end.
    dma_idx = [i for i, r in enumerate(rows) if "gemm_dma_kernel" in r["Kernel_Name"]]
    want = 53 * fwd
    if len(dma_idx) < want + 53 * skip:
        sys.exit("trace too short")
    first = dma_idx[-(want + 53 * skip)]
    end = dma_idx[-53 * skip] if skip else len(rows)
    # extend to the non-conv kernels that follow the last conv of the window
    if skip:
        while end > 0 and "gemm_dma_kernel" not in rows[end - 1]["Kernel_Name"]:
            end -= 1
        j = end
        while j < len(rows) and "gemm_dma_kernel" not in rows[j]["Kernel_Name"]:
            j += 1
        end = min(j, len(rows)) if j - end < 8 else end
    tail = rows[first:end]
    fam = defaultdict(lambda: [0.0, 0])
    for r in tail:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        f = family(r["Kernel_Name"])
        fam[f][0] += d
        fam[f][1] += 1
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) * 1e-6
    busy = 0.0
    cur_s = cur_e = None
    for r in sorted(tail, key=lambda r: int(r["Start_Timestamp"])):
        s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_e is None or s0 > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s0, e0
        else:
            cur_e = max(cur_e, e0)
    busy += cur_e - cur_s
    print(f"{fwd} forwards: {len(tail)} dispatches, wall span {span:.3f} ms "
          f"({span / fwd:.4f} ms/forward), GPU busy (union of kernels) {busy * 1e-6 / fwd:.4f} ms/forward")
    for f, (ms, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"  {f:40s} {ms / fwd:9.4f} ms/forward  {n // fwd:4d} launches/forward  avg {ms / n * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
