#!/bin/bash
# queue delivery: GPU-side cost per dispatch by completion-signal kind (empty kernels, drain
# us per dispatch = GPU time), NVRX_CAPTURE_QUEUE_DIAG 0 (GPU-only HSA signals), 2 (no
# profiling), 3 (amd_signal_t records in device memory).  gpurun_out/r05_qdiag/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_qdiag
mkdir -p "$OUT"
cd "$R"
for rep in 1 2; do
  for d in none 0 2 3; do
    if [ $d = none ]; then
      timeout -k 5 60 ./tools/capture_cost none 20000 > "$OUT/c_$d.json" 2> "$OUT/c_$d.err" || { echo "fail $d"; tail -5 "$OUT/c_$d.err"; exit 1; }
    else
      NVRX_CAPTURE_DELIVERY=queue NVRX_CAPTURE_QUEUE_DIAG=$d timeout -k 5 60 ./tools/capture_cost started 20000 > "$OUT/c_$d.json" 2> "$OUT/c_$d.err" || { echo "fail $d"; tail -5 "$OUT/c_$d.err"; exit 1; }
    fi
    python -c "import json;d=json.load(open('$OUT/c_$d.json'));print('diag $d launch', d['launch_us_per_dispatch'], 'drain', d['drain_us_per_dispatch'])"
  done
done
