# Chained folds, url selections, event order: their GPU tests, the multi-term
# config tests, then the C3 / C4 legs of the bench.
set -o pipefail
mkdir -p gpurun_out/chain
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
  -k "chained or urlselection or long_bitmap or j5_side or forced_join or null_stats" > gpurun_out/chain/t1.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_java_sequence.py tests/test_events.py -x -v \
  --timeout 300 --timeout-method thread -k "c3_shard or c4_batch or java or event" > gpurun_out/chain/t2.log 2>&1 || exit $?
timeout -k 10 1100 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/chain/legs.json 2> gpurun_out/chain/legs.err || exit $?
