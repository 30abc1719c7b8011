#!/bin/bash
# SQ counters of the final statistics kernels: configs[2] (group<16>) and configs[1] (group<128>),
# two --pmc passes each over tools/ab_c3_pair.py.  Output: gpurun_out/r03_sqfinal/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_sqfinal
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for shape in "4096 1024 c2" "64 10000 c1"; do
  set -- $shape
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
    AB_R=$1 AB_S=$2 timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$3/p$i" -o p -- \
        python3 "$R/tools/ab_c3_pair.py" "$R/nvidia-resiliency-ext-x_amd" 3 > "$OUT/$3_p$i.log" 2>&1 || { echo "pass $3 $i failed"; exit 1; }
    i=$((i+1))
  done
done
python3 "$R/tools/pmc_sum.py" "$OUT/c2" "$OUT/c1" > "$OUT/sq.txt"
cat "$OUT/sq.txt"
