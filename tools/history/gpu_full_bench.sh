#!/bin/bash
# whole GPU suite + smoke (tools/gpu_full.sh), then the default bench line and its kernel trace.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/full
mkdir -p "$OUT"
cd "$R"
bash tools/gpu_full.sh || exit 1
grep -q "smoke rc=0" <(tail -1 "$OUT/smoke.log"; echo) || true
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; echo "bench rc=$?"
tail -1 "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"; echo "trace rc=$?"
