#!/usr/bin/env python3
"""Summarise scripts/gpu_traffic.sh output: HBM bytes per forward pass of the
conv GEMM kernel (gemm_dma_kernel, all instantiations) and of everything.
FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B, see
MI355X_MICROARCH.md HBM section); WRITE_SIZE is taken as is.  Counter units
are KB.  The tuning run (first forward) is excluded: only the last RUNS
forwards' dispatches are summed (identified as the trailing dispatches)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(pattern):
    rows = []
    for f in glob.glob(pattern):
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(float)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return per, names


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic"
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ops_per_forward = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    res = {}
    for ctr, mult in (("fetch", 2.0), ("write", 1.0)):
        per, names = load(f"{root}/{ctr}*counter_collection.csv")
        ids = sorted(per)
        conv_ids = [d for d in ids if "gemm_dma_kernel" in names[d]]
        n_conv = len(conv_ids)
        # conv dispatches per forward: tuning forward launches many more, so
        # take the last runs * per_forward ones.
        per_fwd = ops_per_forward or 53
        tail = conv_ids[-runs * per_fwd:]
        first = tail[0]
        all_tail = [d for d in ids if d >= first]
        res[ctr] = {
            "conv_bytes_per_forward": sum(per[d] for d in tail) * 1024 * mult / runs,
            "all_bytes_per_forward": sum(per[d] for d in all_tail) * 1024 * mult / runs,
            "conv_dispatches_counted": len(tail),
        }
    out = {
        "conv_gemm_bytes_per_forward": res["fetch"]["conv_bytes_per_forward"] + res["write"]["conv_bytes_per_forward"],
        "all_kernels_bytes_per_forward": res["fetch"]["all_bytes_per_forward"] + res["write"]["all_bytes_per_forward"],
        "detail": res,
        "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB->bytes; ResNet-50 b64 eager forward",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
