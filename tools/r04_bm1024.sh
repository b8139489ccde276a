# Bitmap threshold nurls/1024 instead of /256: C3 / C4 legs and the chain path counters.
set -o pipefail
mkdir -p gpurun_out/bm1024
YRWI_BM_DIV=1024 YRWI_LIB=$PWD/yacy_search_server_amd/libyrwi_cprof.so timeout -k 10 300 python3 -u tools/chain_prof.py C3 3 1 \
  > gpurun_out/bm1024/cprof.json 2> gpurun_out/bm1024/cprof.err || exit $?
YRWI_BM_DIV=1024 timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/bm1024/legs.json 2> gpurun_out/bm1024/legs.err || exit $?
