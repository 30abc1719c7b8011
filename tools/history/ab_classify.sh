#!/bin/bash
# Ragged / record-stream GPU tests, then the configs[3] record-stream statistics under a
# kernel trace (classify_count / classify_scatter timings); output under gpurun_out/cls/.
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/cls; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 120 python tools/ab_zipf.py 6 > $O/ab.txt 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o z -- python3 $GRAFT_REPO_ROOT/tools/ab_zipf.py 4 > $O/trace.log 2>&1
echo ok
