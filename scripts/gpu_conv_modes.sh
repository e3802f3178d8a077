#!/bin/bash
# One conv layer through the device graph under forced kernel choices
# (RTENHIP_PW_VALU), each step with its own time limit.  usage: SHAPE="N C H W O k s p [clip]" MODES="0 316 332"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for m in $MODES; do
  RTENHIP_PW_VALU=$m timeout -k 10 120 python3 rten-fork_amd/tools/conv_graph_time.py $SHAPE || exit 1
done
