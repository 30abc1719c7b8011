# lean vs fast stats body at every FULL segment length (production generator data) -> gpurun_out/mball/
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/mball; mkdir -p $O
B=$GRAFT_REPO_ROOT/tools/build/mb_c3
timeout -k 10 120 $B 4096 s 16 5 > $O/pl16.log 2>&1
timeout -k 10 120 $B 2048 s 32 5 > $O/pl32.log 2>&1
timeout -k 10 120 $B 1024 s 64 5 > $O/pl64.log 2>&1
timeout -k 10 120 $B 128 s 128 10 > $O/pl128.log 2>&1
echo ok
