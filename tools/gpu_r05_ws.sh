#!/bin/bash
# Round 5: the warp-specialised bucketing kernel (records.hip,
# records_bucket_ws_kernel; NVRX_RB_WS=RWxSW) against the shipped one on configs[3], interleaved,
# with the statistics of every variant compared bit for bit against the shipped kernel's.
# gpurun_out/r05_ws/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_ws${TAG}
mkdir -p "$OUT"
cd "$R"
: > "$OUT/ab.log"
for rep in $(seq 1 ${REPS:-2}); do
  for ws in ${SPLITS:-0 4x12 6x10 8x8}; do
    NVRX_RB_WS=$ws AB_DUMP="$OUT/dump_$ws.pt" timeout -k 10 120 python -u tools/ab_zipf.py ${NCALL:-10} >> "$OUT/ab.log" 2> "$OUT/err_$ws.log" || { echo "fail $ws"; tail -20 "$OUT/err_$ws.log"; exit 1; }
    tail -1 "$OUT/ab.log"
  done
done
python - "$OUT" <<'PY'
import sys, torch, glob, os
d = sys.argv[1]
ref = torch.load(os.path.join(d, "dump_0.pt"))
for f in sorted(glob.glob(os.path.join(d, "dump_*.pt"))):
    x = torch.load(f)
    same = all(torch.equal(x[k].view(torch.int32), ref[k].view(torch.int32)) for k in ref)
    print(os.path.basename(f), "bit-identical to the shipped kernel:", same)
PY
