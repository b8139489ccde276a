# Count-first chained folds: the chained-fold GPU tests (forced count-first included),
# the path counters, then the C3 / C4 legs.
set -o pipefail
mkdir -p gpurun_out/cf
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread \
  -k "chained or urlselection or long_bitmap or forced_join or c3_shard or c4_batch or j5" > gpurun_out/cf/t.log 2>&1 || exit $?
YRWI_LIB=$PWD/yacy_search_server_amd/libyrwi_cprof.so timeout -k 10 300 python3 -u tools/chain_prof.py C3 3 1 \
  > gpurun_out/cf/cprof.json 2> gpurun_out/cf/cprof.err || exit $?
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/cf/legs.json 2> gpurun_out/cf/legs.err || exit $?
