# Chained folds: their GPU tests first (new kernels: stop at the first failure),
# then the multi-term config tests, then the C3 / C4 legs of the bench.
set -o pipefail
mkdir -p gpurun_out/chain
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
  -k "chained or long_bitmap or j5_side or forced_join or null_stats" > gpurun_out/chain/t1.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "c3_shard or c4_batch" > gpurun_out/chain/t2.log 2>&1 || exit $?
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4 --no-cpu --latency 0 --leg-latency 0 \
  > gpurun_out/chain/legs.json 2> gpurun_out/chain/legs.err || exit $?
