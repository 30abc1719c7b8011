#!/bin/bash
# configs[3] record-stream kernels: SQ counters (wave-cycle split, LDS activity / conflicts,
# instruction mix) in two --pmc passes of 8 SQ counters each; output under gpurun_out/pmc_sq/.
set -e
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out/pmc_sq}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export AB_R=${AB_R:-16384}
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
B="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES"
i=0
for grp in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- \
      python3 "$R/tools/ab_zipf.py" 2 > "$OUT/p$i.log" 2>&1
done
echo done
