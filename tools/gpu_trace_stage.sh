#!/bin/bash
# kernel traces of configs[3] record statistics under staging settings ("KB COLD" pairs).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/trace_stage
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  set -- $v
  NVRX_RB_STAGE_KB=$1 NVRX_RB_COLD=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/s$1_c$2" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/s$1_c$2.log" 2>&1 || exit 1
done
echo done
