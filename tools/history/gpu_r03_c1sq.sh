#!/bin/bash
# configs[1] statistics: block kernel (tree) vs lean<128> (tools/ab_pkg), interleaved; then SQ
# counters of both (two --pmc passes each).  Output: gpurun_out/r03_c1sq/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_c1sq
mkdir -p "$OUT"
cd "$R"
export AB_R=64 AB_S=10000
timeout -k 10 120 tools/build/mb_c2 > "$OUT/mb_c2.log" 2>&1 || exit 1; grep cfg1 "$OUT/mb_c2.log"
for i in 1; do
  timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/tools/ab_pkg" 50 2>&1 | grep ms= || exit 1
  timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/nvidia-resiliency-ext-x_amd" 50 2>&1 | grep ms= || exit 1
done | tee "$OUT/ab.log"
cd /tmp && export TMPDIR=/tmp
for pkg in tools/ab_pkg nvidia-resiliency-ext-x_amd; do
  tag=$(basename $pkg); mkdir -p "$OUT/$tag"
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$tag/p$i" -o p -- python3 "$R/tools/ab_c3_pair.py" "$R/$pkg" 3 > "$OUT/$tag/p$i.log" 2>&1 || { echo "pass $tag $i failed"; exit 1; }
    i=$((i+1))
  done
done
python3 "$R/tools/pmc_sum.py" "$OUT/ab_pkg" "$OUT/nvidia-resiliency-ext-x_amd" > "$OUT/sq.txt"
cat "$OUT/sq.txt"
