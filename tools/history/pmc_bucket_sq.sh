#!/bin/bash
# records_bucket_kernel counters, this tree and _ab_old: SQ wave-cycle split and LDS, the
# instruction mix, and TA/TD/TCP (address path, translation) -- one --pmc pass per group.
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out/pmc_bucket}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
G2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES"
G3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
for tree in new old; do
  d=$R; [ $tree = old ] && d=$R/_ab_old
  i=0
  for grp in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${tree}_p$i" -o p -- \
        python3 "$d/tools/ab_zipf.py" 2 > "$OUT/${tree}_p$i.log" 2>&1 || { echo "$tree pass $i failed"; tail -3 "$OUT/${tree}_p$i.log"; }
  done
done
echo done
