#!/bin/bash
# Kernel-traced convbench under variant builds (rten-fork_amd/var_*/), on
# ResNet-50 layer shapes; prints the median DMA-kernel time per (variant,
# config, shape).  usage: LIBS="t2 t4" CFGS=d0,d1 bash scripts/gpu_var.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/var
SH=${SH:-"--shape 64,1024,14,14,256,1,1,0 --shape 64,256,14,14,256,3,1,1 --shape 64,512,7,7,512,3,1,1 --shape 64,64,56,56,256,1,1,0 --shape 64,64,56,56,64,3,1,1 --shape 64,2048,7,7,512,1,1,0"}
for v in $LIBS; do
  RTENHIP_LIB=$PWD/rten-fork_amd/$v/librten_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/var -o $v -- python3 rten-fork_amd/tools/convbench.py --iters 6 --cfgs ${CFGS:-d0,d1,d2,d3} $SH > gpurun_out/var_$v.log 2>&1 || { echo $v failed; tail gpurun_out/var_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, os, re
for v in os.environ["LIBS"].split():
    rows = list(csv.DictReader(open(f'gpurun_out/var/{v}_kernel_trace.csv')))
    out = []
    for r in rows:
        n = r['Kernel_Name']
        if 'gemm_dma' not in n: continue
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
        t = re.search(r'gemm_dma_kernel<([^>]*)>', n).group(1)
        key = (t, r['Grid_Size_X'])
        if out and out[-1][0] == key: out[-1][1].append(d)
        else: out.append([key, [d]])
    print("variant", v)
    for k, vals in out:
        if len(vals) > 2: print(f"  <{k[0]:45s}> blocks={int(k[1])//int(rows[0]['Workgroup_Size_X'] or 256):6d} med={sorted(vals)[len(vals)//2]:7.1f}us")
PY
