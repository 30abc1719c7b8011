#!/bin/bash
# round-2 profiles: the default bench under --kernel-trace --stats, the C2 stats kernel's HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes), and configs[2]'s stats kernel counters.
R=$GRAFT_REPO_ROOT
bash "$R/tools/profile_round.sh" || { echo "profile_round failed"; exit 1; }
export AB_R=4096
OUT=$R/gpurun_out/pmc_c3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- python3 "$R/tools/ab_c3.py" 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/tools/ab_c3.py" 5 > "$OUT/trace.log" 2>&1
echo ok
