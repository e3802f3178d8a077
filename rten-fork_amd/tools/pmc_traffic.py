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
    for f in glob.glob(pattern, recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(float)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return per, names


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    root = args[0] if len(args) > 0 else "gpurun_out/traffic"
    runs = int(args[1]) if len(args) > 1 else 2
    ops_per_forward = int(args[2]) if len(args) > 2 else 0
    if "--marker" in sys.argv:
        return marker_mode(root, runs)
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


def marker_mode(root, runs):
    """Every dispatch after the marker fill of tools/model_once.py, per
    forward, by kernel family."""
    res = {}
    fam_all = defaultdict(float)
    for ctr, mult in (("fetch", 2.0), ("write", 1.0)):
        per, names = load(f"{root}/**/{ctr}*counter_collection.csv")
        ids = sorted(per)
        # the torch fill (at::native kernel) of model_once.py; the forwards
        # themselves launch librten_hip kernels and HIP's own memset kernels
        last_marker = max((d for d in ids if "at::" in names[d]), default=-1)
        tail = [d for d in ids if d > last_marker]
        fam = defaultdict(float)
        for d in tail:
            k = names[d].replace("(anonymous namespace)::", "")
            k = k.split("(")[0].split("<")[0].replace("void ", "").strip()
            fam[k] += per[d] * 1024 * mult / runs
            fam_all[k] += per[d] * 1024 * mult / runs
        res[ctr] = {"bytes_per_forward": sum(fam.values()), "dispatches_per_forward": len(tail) / runs,
                    "by_kernel": dict(sorted(fam.items(), key=lambda kv: -kv[1]))}
    out = {
        "all_kernels_bytes_per_forward": res["fetch"]["bytes_per_forward"] + res["write"]["bytes_per_forward"],
        "by_kernel": dict(sorted(fam_all.items(), key=lambda kv: -kv[1])),
        "detail": res,
        "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB->bytes; eager forwards after the tuning run",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
