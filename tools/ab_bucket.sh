#!/bin/bash
# A/B of record-bucketing block shapes on configs[3] (tools/ab_zipf.py), with the LDS stash:
# NVRX_RB_WAVES waves per block, NVRX_RB_BPC blocks per CU (LDS padding; the stash takes what
# the padding leaves).  Three interleaved rounds; output lines under gpurun_out/bucket/.
cd $GRAFT_REPO_ROOT
O=gpurun_out/bucket; mkdir -p $O
for i in 1 2 3; do
  for v in "NVRX_RB_BPC=1" "NVRX_RB_BPC=2" "NVRX_RB_WAVES=8" "NVRX_RB_WAVES=8 NVRX_RB_BPC=2" "NVRX_RB_WAVES=16"; do
    env $v timeout -k 10 120 python tools/ab_zipf.py 6 2>/dev/null | tail -1 >> $O/ab.txt || exit 1
  done
done
echo ok
