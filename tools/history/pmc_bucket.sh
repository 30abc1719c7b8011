#!/bin/bash
# HBM traffic of the record bucketing kernel (FETCH_SIZE, WRITE_SIZE in KB; gfx950: FETCH x2).
OUT=${OUT:-$GRAFT_REPO_ROOT/gpurun_out/pmc_b}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  AB_R=${AB_R:-4096} timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- python3 "$GRAFT_REPO_ROOT/tools/ab_zipf.py" 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; }
  i=$((i+1))
done
