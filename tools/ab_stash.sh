set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/stash; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2 3; do
  NVRX_RB_STASH=0 timeout -k 10 120 python tools/ab_zipf.py 6 2>/dev/null | tail -1 >> $O/ab.txt
  timeout -k 10 120 python tools/ab_zipf.py 6 2>/dev/null | tail -1 >> $O/ab.txt
done
echo ok
