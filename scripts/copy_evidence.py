#!/usr/bin/env python3
"""Copy a gpu_evidence.sh run (gpurun_out/prof_TAG) into profiles/ as the
round's evidence: per-forward rocprof summaries and kernel stats, PMC traffic
summaries and per-op reports, each stamped with the last commit that changed
the product sources (what bench.py's rocprof / traffic fields compare with).
Usage: scripts/copy_evidence.py TAG ROUND   e.g. r6b r6"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import SOURCE_PATHS  # noqa: E402

tag, rnd = sys.argv[1], sys.argv[2]
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
git = lambda *a: subprocess.run(["git", "-C", ROOT] + list(a), capture_output=True, text=True).stdout.strip()
commit = git("log", "-1", "--format=%h", "--", *SOURCE_PATHS)
head = git("rev-parse", "--short", "HEAD")
stamp = f"{commit} (last source change; taken at {head}; scripts/gpu_evidence.sh {tag})"
dst = os.path.join(ROOT, "profiles")
for f in sorted(os.listdir(src)):
    p = os.path.join(src, f)
    if f.endswith("_per_forward.txt"):
        body = open(p).read()
        open(os.path.join(dst, f"{rnd}_rocprof_{f}"), "w").write(
            f"# commit {stamp}: timed replays; tools/rocprof_per_forward.py\n" + body)
    elif f.endswith("_kernel_stats.csv"):
        shutil.copy(p, os.path.join(dst, f"{rnd}_rocprof_{f}"))
    elif f.startswith("pmc_traffic_") and f.endswith(".json"):
        js = json.load(open(p))
        js["commit"] = stamp
        json.dump(js, open(os.path.join(dst, f"{rnd}_{f}"), "w"), indent=1)
    elif f.startswith("report_") and f.endswith(".txt"):
        body = "".join(l for l in open(p) if "amdgpu.ids" not in l)
        open(os.path.join(dst, f"{rnd}_{f}"), "w").write(f"# commit {stamp}\n" + body)
print("copied", src, "->", dst, "as", rnd, "at", stamp)
