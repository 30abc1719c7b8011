#!/bin/bash
# The round's measurement on one MI355X (run through gpurun): the default bench line, its
# rocprofv3 kernel-trace summary, the configs[1] statistics kernel's FETCH_SIZE / WRITE_SIZE
# passes, the configs[2] kernel's, and the configs[3] per-kernel traffic -- each --pmc counter
# group in its own run (MI355X_MICROARCH.md, HBM / rocprofv3 section).  Output:
# gpurun_out/${PROF_TAG:-prof}/; tools/pmc_json.py turns the passes into profiles/pmc_*.json.
# STEPS selects what runs (default "bench trace c2 c3 zipf").
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PROF_TAG:-prof}
STEPS=${STEPS:-"bench trace c2 c3 zipf"}
mkdir -p "$OUT"
has() { [[ " $STEPS " == *" $1 "* ]]; }
cd "$R"
if has bench; then
  timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  tail -1 "$OUT/bench.json" | cut -c1-300
fi
cd /tmp && export TMPDIR=/tmp
if has trace; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
      python3 "$R/bench.py" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
  echo trace done
fi
if has c2; then  # configs[1]: the headline's statistics kernel
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/c2_$c" -o p -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-latency4096 --no-zipf --no-cpu-baseline \
        > "$OUT/c2_$c.log" 2>&1
  done
  echo c2 done
fi
if has c3; then  # configs[2]: 4096 x 2048 x 1024
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3_trace" -o t -- \
      python3 "$R/tools/ab_c3_pair.py" "$R/nvidia-resiliency-ext-x_amd" 5 > "$OUT/c3_trace.log" 2>&1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/c3_$c" -o p -- \
        python3 "$R/tools/ab_c3_pair.py" "$R/nvidia-resiliency-ext-x_amd" 3 > "$OUT/c3_$c.log" 2>&1
  done
  echo c3 done
fi
if has zipf; then  # configs[3]: 16,384 Zipf record streams
  export AB_R=${AB_R:-16384}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/zipf_trace" -o t -- \
      python3 "$R/tools/ab_zipf.py" 3 > "$OUT/zipf_trace.log" 2>&1
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo "$grp" | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/zipf_$tag" -o p -- \
        python3 "$R/tools/ab_zipf.py" 2 > "$OUT/zipf_$tag.log" 2>&1
  done
  echo zipf done
fi
