#!/bin/bash
# pack_a rows-per-workgroup sweep (RTENHIP_PACK_RB) on BERT b32: per-forward
# pack_a time under rocprofv3 and the bench line.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/packrb; mkdir -p $O
for rb in 16 32 64 128; do
  RTENHIP_PACK_RB=$rb timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof_$rb -o run --output-format csv -- python3 bench.py --model bert --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$rb.log 2>&1 || { echo rocprof $rb failed; tail $O/prof_$rb.log; exit 1; }
  echo "== RB=$rb"; python3 rten-fork_amd/tools/rocprof_per_forward.py $(find $O/prof_$rb -name run_kernel_trace.csv) 10 156 | grep -E "pack_a|GPU busy"
done
