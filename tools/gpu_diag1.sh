#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/diag1
mkdir -p "$OUT"
cd "$R"
export NVRX_CAPTURE_DEBUG=1
timeout -k 10 120 python tools/diag_capture.py > "$OUT/ready.log" 2>&1; echo "rc=$?" >> "$OUT/ready.log"
DIAG_BUFSIZE=8192 timeout -k 10 120 python tools/diag_capture.py > "$OUT/drain.log" 2>&1; echo "rc=$?" >> "$OUT/drain.log"
NVRX_CAPTURE_WATERMARK=4096 DIAG_BUFSIZE=8192 timeout -k 10 120 python tools/diag_capture.py > "$OUT/drain_wm.log" 2>&1; echo "rc=$?" >> "$OUT/drain_wm.log"
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 tests/func/ddp_straggler.py --iters 61 --report-iter-interval 20 > "$OUT/ddp.out" 2> "$OUT/ddp.err"; echo "rc=$?" >> "$OUT/ddp.out"
grep -h "available\|captured\|nvrx\|rc=" "$OUT"/*.log "$OUT/ddp.out"
