#!/bin/bash
# batched-load scores kernel: the whole GPU suite, then the configs[1] report (bench value leg)
# this tree vs _ab_old, interleaved.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_scores
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; tail -3 "$OUT/pytest.log"
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    timeout -k 10 200 python bench.py --no-latency4096 --no-zipf --no-cpu-baseline --steps 200 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$tree', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g' % d['value'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/bench.py" --no-latency4096 --no-zipf --no-cpu-baseline --steps 50 > "$OUT/trace.log" 2>&1
grep -h "scores_kernel" "$OUT"/trace/*kernel_stats.csv | cut -c1-160
