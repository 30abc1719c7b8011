#!/bin/bash
# Counter passes over the C3 stats kernel (tools/ab_c3.py); one --pmc group per pass.
set -e
OUT=${OUT:-$GRAFT_REPO_ROOT/gpurun_out/pmc_c3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  AB_R=${AB_R:-1024} timeout -k 10 180 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p -- python3 "$GRAFT_REPO_ROOT/tools/ab_c3.py" 2 > "$OUT/p$i.log" 2>&1 || echo "pass $i failed" >> "$OUT/fail.txt"
  i=$((i+1))
done
