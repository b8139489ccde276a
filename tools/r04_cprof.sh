# k_chain path counters (profiling build) for C3 at the default bitmap threshold and at
# nurls/1024, then the C3 leg at nurls/1024.
set -o pipefail
mkdir -p gpurun_out/cprof
YRWI_LIB=$PWD/yacy_search_server_amd/libyrwi_cprof.so timeout -k 10 300 python3 -u tools/chain_prof.py C3 3 1 \
  > gpurun_out/cprof/c3_bm256.json 2> gpurun_out/cprof/c3_bm256.err || exit $?
YRWI_BM_DIV=1024 YRWI_LIB=$PWD/yacy_search_server_amd/libyrwi_cprof.so timeout -k 10 300 python3 -u tools/chain_prof.py C3 3 1 \
  > gpurun_out/cprof/c3_bm1024.json 2> gpurun_out/cprof/c3_bm1024.err || exit $?
YRWI_BM_DIV=1024 timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/cprof/legs_bm1024.json 2> gpurun_out/cprof/legs_bm1024.err || exit $?
