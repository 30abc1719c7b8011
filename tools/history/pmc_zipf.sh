#!/bin/bash
# Counter passes over the configs[3] stats kernels (tools/ab_zipf.py, AB_R ranks).
OUT=${OUT:-$GRAFT_REPO_ROOT/gpurun_out/pmc_z}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  AB_R=${AB_R:-4096} timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- python3 "$GRAFT_REPO_ROOT/tools/ab_zipf.py" 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
  i=$((i+1))
done
