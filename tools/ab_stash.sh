#!/bin/bash
# Record-bucketing LDS stash A/B on configs[3] (tools/ab_zipf.py), after the records tests:
# NVRX_RB_STASH=0 no stash, =1 stash placed before the rest, default stash interleaved with
# the rest's loads; NVRX_RB_WAVES=8 the 8-wave block.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/stash; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2 3; do
  for v in "NVRX_RB_STASH=0" "NVRX_RB_STASH=1" "NVRX_RB_STASH=2" "NVRX_RB_WAVES=8"; do
    env $v timeout -k 10 120 python tools/ab_zipf.py 6 2>/dev/null | tail -1 >> $O/ab.txt
  done
done
echo ok
