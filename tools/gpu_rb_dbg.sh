#!/bin/bash
# timing experiment: which stores of the bucket scatter cost (NVRX_RB_DBG skips some; wrong output)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for v in 0 1 2 3; do
  NVRX_RB_DBG=$v timeout -s KILL 100 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/rbdbg/v${v}_$i" -o t -- python3 "$R/tools/ab_zipf.py" 5 > /dev/null 2>&1
  echo -n "dbg=$v: "; grep -h "records_bucket" "$R"/gpurun_out/rbdbg/v${v}_$i/*kernel_stats.csv | cut -d, -f4
done
done
