#!/bin/bash
# Round-3 starting point, default build: configs[3] per-kernel trace + FETCH_SIZE / WRITE_SIZE
# passes (tools/pmc_zipf_traffic.sh), then configs[2] lean<16> SIMD-utilisation counters
# (GRBM_GUI_ACTIVE for chip cycles next to SQ wave/VALU cycles).  Output: gpurun_out/r03_base/.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_base
mkdir -p "$OUT"
OUT=$OUT/zipf bash "$R/tools/pmc_zipf_traffic.sh"
cd /tmp && export TMPDIR=/tmp
export AB_R=4096
i=0
for grp in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/c3_p$i" -o p -- \
      python3 "$R/tools/ab_c3.py" 2 > "$OUT/c3_p$i.log" 2>&1 || echo "c3 pass $i failed"
  i=$((i+1))
done
echo done
