#!/usr/bin/env python3
"""Copy a GPU evidence run (scripts/gpu_evidence.sh -> gpurun_out/prof_TAG)
into profiles/ as {round}_rocprof_* / {round}_pmc_traffic_* / {round}_report_*,
stamped with the commit the run was made from (the GPU box gets no .git, so
the commit is given here): a "commit" field in the JSON summaries, a first
line in the text ones.
usage: stamp_profiles.py TAG ROUND COMMIT"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    tag, rnd, commit = sys.argv[1:4]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    for f in sorted(os.listdir(src)):
        p = os.path.join(src, f)
        if f.startswith("pmc_traffic_") and f.endswith(".json"):
            js = json.load(open(p))
            js["commit"] = commit
            out = os.path.join(dst, f"{rnd}_{f}")
            json.dump(js, open(out, "w"), indent=1)
        elif f.endswith("_per_forward.txt") or f.endswith("_kernel_stats.csv") or f.startswith("report_"):
            name = f if f.startswith("report_") else "rocprof_" + f
            out = os.path.join(dst, f"{rnd}_{name}")
            body = open(p).read()
            if f.endswith(".csv"):
                shutil.copy(p, out)
                open(out + ".commit", "w").write(commit + "\n")
                print(out)
                continue
            open(out, "w").write(f"# commit {commit} (scripts/gpu_evidence.sh {tag})\n" + body)
        else:
            continue
        print(out)


if __name__ == "__main__":
    main()
