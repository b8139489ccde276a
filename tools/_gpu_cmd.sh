set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards_loopback.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest_lb.log 2>&1
