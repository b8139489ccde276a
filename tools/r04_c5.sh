# C5 legs (authority k_reduce) and the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/c5/t.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C5,C4 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/c5/legs.json 2> gpurun_out/c5/legs.err || exit $?
