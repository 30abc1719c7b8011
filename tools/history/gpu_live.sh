set -e
mkdir -p gpurun_out/live
timeout -k 10 400 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_live.py -x -v --timeout 300 --timeout-method thread > gpurun_out/live/pytest.log 2>&1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 400 python -u tools/live_gpt2.py --out gpurun_out/live/live_gpt2.json > gpurun_out/live/live.log 2>&1
echo ok
