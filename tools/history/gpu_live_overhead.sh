# capture-overhead breakdown of the live GPT-2 loop (configs[4]); logs under gpurun_out/live/
set -e
mkdir -p gpurun_out/live
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
L="python -u tools/live_gpt2.py --steps 40 --base-steps 20"
MASTER_PORT=29541 timeout -k 10 300 $L --out gpurun_out/live/o_full.json > gpurun_out/live/o_full.log 2>&1
MASTER_PORT=29542 NVRX_CAPTURE_WATERMARK=6291456 timeout -k 10 300 $L --out gpurun_out/live/o_wm6m.json > gpurun_out/live/o_wm6m.log 2>&1
MASTER_PORT=29543 NVRX_CAPTURE_WATERMARK=131072 timeout -k 10 300 $L --out gpurun_out/live/o_wm128k.json > gpurun_out/live/o_wm128k.log 2>&1
echo ok
