#!/bin/bash
# configs[2] stats kernel (lean<16>) SQ counters: instruction mix and wave-cycle split, two
# --pmc passes over tools/ab_c3.py; output under gpurun_out/pmc_c3_sq/.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_c3_sq
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export AB_R=4096
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- python3 "$R/tools/ab_c3.py" 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo ok
