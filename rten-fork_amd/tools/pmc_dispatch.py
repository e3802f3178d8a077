#!/usr/bin/env python3
"""Per-dispatch view of one rocprofv3 --pmc pass over tools/model_once.py:
every librten_hip dispatch after the marker of the LAST eager forward, in
order, with its duration, MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
1024 SIMDs x GRBM_GUI_ACTIVE / 8 cycles) and the wave-state split
(SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES).
usage: pmc_dispatch.py DIR [forwards]   (forwards: eager forwards after the marker, default 2)"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    fw = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    disp = defaultdict(dict)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            i = int(r["Dispatch_Id"])
            d = disp[i]
            d["name"] = r["Kernel_Name"]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if "Start_Timestamp" in r:
                d["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    ids = sorted(disp)
    # The marker is model_once's torch fill; the runtime's own copy / fill
    # kernels (__amd_rocclr_*, e.g. BERT's int32 inputs) belong to the forwards.
    def ours(i):
        return "rtenhip" in disp[i]["name"] or "__amd_rocclr" in disp[i]["name"]

    mark = max((i for i in ids if not ours(i)), default=-1)
    after = [i for i in ids if i > mark and ours(i)]
    per = len(after) // fw if fw else len(after)
    last = after[-per:]
    print(f"{len(after)} dispatches after the marker, {per} per forward; the last forward:")
    print(f"{'#':>3} {'us':>8} {'mfma':>6} {'wait':>6} {'winst':>6} {'active':>6}  kernel")
    for k, i in enumerate(last):
        d = disp[i]
        cyc = d.get("GRBM_GUI_ACTIVE", 0) / 8
        mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * cyc) if cyc else 0
        wc = d.get("SQ_WAVE_CYCLES", 0)
        w = d.get("SQ_WAIT_ANY", 0) / wc if wc else 0
        wi = d.get("SQ_WAIT_INST_ANY", 0) / wc if wc else 0
        ac = d.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else 0
        name = d["name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
        print(f"{k:3d} {d.get('dur', 0):8.1f} {mf:6.3f} {w:6.2f} {wi:6.2f} {ac:6.2f}  {name}")


if __name__ == "__main__":
    main()
