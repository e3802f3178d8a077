#!/bin/bash
# Kernel-trace the DMA GEMM under experiment builds on a K sweep.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/exptrace
SH=${SH:-"--shape 64,256,14,14,256,1,1,0 --shape 64,512,14,14,256,1,1,0 --shape 64,1024,14,14,256,1,1,0 --shape 64,2048,14,14,256,1,1,0 --shape 64,4096,14,14,256,1,1,0"}
for m in ${MODES:-0 4}; do
  RTENHIP_LIB=$PWD/rten-fork_amd/exp$m/librten_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/exptrace -o k$m -- python3 rten-fork_amd/tools/convbench.py --cfgs ${CFGS:-d2,d3} $SH > gpurun_out/exptrace_k$m.log 2>&1 || { echo m$m failed; tail gpurun_out/exptrace_k$m.log; exit 1; }
done
python3 - <<'PY'
import csv, os
for m in os.environ.get("MODES", "0 4").split():
    rows = list(csv.DictReader(open(f'gpurun_out/exptrace/k{m}_kernel_trace.csv')))
    out = []
    for r in rows:
        n = r['Kernel_Name']
        if 'gemm_dma' not in n: continue
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
        key = (n[:75], r['Grid_Size_X'])
        if out and out[-1][0] == key: out[-1][1].append(d)
        else: out.append([key, [d]])
    print("mode", m)
    for k, v in out:
        if len(v) > 1: print(f"  {k[0]:75s} blocks={int(k[1])//256:6d} med={sorted(v)[len(v)//2]:7.1f}us")
PY
