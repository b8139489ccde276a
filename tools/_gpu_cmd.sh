set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
ls /dev/shm > gpurun_out/shm_after.txt && \
timeout -k 10 300 python -u bench.py --no-cpu --legs none --latency 0 --steps 400 --warmup 40 > gpurun_out/bench.json 2> gpurun_out/bench.err
