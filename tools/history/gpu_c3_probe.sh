# C3 probe: launch-shape microbenchmark (production data) + production kernel timing +
# instruction-count counters of the C3 stats kernel (R=1024 for speed).  -> gpurun_out/c3probe/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c3probe
mkdir -p $O
cd $R
timeout -k 10 200 tools/build/mb_c3 4096 s > $O/mb_c3s.log 2>&1
timeout -k 10 200 python tools/ab_c3.py 5 > $O/ab_c3.log 2>&1
cd /tmp && export TMPDIR=/tmp
AB_R=1024 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $O/p0 -o p -- python3 $R/tools/ab_c3.py 2 > $O/p0.log 2>&1
AB_R=1024 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d $O/p1 -o p -- python3 $R/tools/ab_c3.py 2 > $O/p1.log 2>&1
echo ok
