#!/usr/bin/env python3
"""Summarise scripts/gpu_pmc2.sh output for the gemm_dma_kernel dispatches:
per-dispatch averages, effective clock, MFMA busy fraction per SIMD, wave
state split.  usage: pmc_layer.py DIR TAG"""
import csv
import glob
import sys
from collections import defaultdict

d, tag = sys.argv[1], sys.argv[2]
vals = defaultdict(float)
dur = []
for f in sorted(glob.glob(f"{d}/{tag}_*_counter_collection.csv")):
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "gemm_dma_kernel" not in r["Kernel_Name"]:
            continue
        disp[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        disp[r["Dispatch_Id"]]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(disp, key=int)[1:]  # drop the first (cold) dispatch
    for k in set().union(*[disp[i].keys() for i in ids]):
        vals[k] = sum(disp[i].get(k, 0) for i in ids) / len(ids)
t = vals["_dur"]
clk = vals["GRBM_GUI_ACTIVE"] / 8 / t / 1e9 if t else 0
cyc = vals["GRBM_GUI_ACTIVE"] / 8
print(f"{tag}: {t*1e6:.1f} us/dispatch, effective clock {clk:.2f} GHz, waves {vals['SQ_WAVES']:.0f}")
print(f"  MFMA busy / (1024 SIMDs x kernel cycles) = {vals['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.3f}")
wc = vals["SQ_WAVE_CYCLES"]
if wc:
    print(f"  wave time: wait_any {vals['SQ_WAIT_ANY']/wc:.2f}  wait_inst {vals['SQ_WAIT_INST_ANY']/wc:.2f}  "
          f"active {vals['SQ_ACTIVE_INST_ANY']/wc:.2f}; avg waves/SIMD resident {wc*4/(1024*cyc):.2f}")
m = vals["SQ_INSTS_MFMA"]
if m:
    print("  per MFMA: " + "  ".join(f"{k[9:]}={vals[k]/m:.2f}" for k in
          ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM")))
    print(f"  wait_inst_lds/wave_cycles {vals['SQ_WAIT_INST_LDS']/max(wc,1):.3f}")
