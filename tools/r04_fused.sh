# Fused probe + chain (matches in LDS) and k_hostcount: the whole GPU suite, the
# chain path counters, then the C3 / C4 / C5 legs.
set -o pipefail
mkdir -p gpurun_out/fused
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/fused/t.log 2>&1 || exit $?
YRWI_LIB=$PWD/yacy_search_server_amd/libyrwi_cprof.so timeout -k 10 300 python3 -u tools/chain_prof.py C3 3 1 \
  > gpurun_out/fused/cprof.json 2> gpurun_out/fused/cprof.err || exit $?
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4,C5 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/fused/legs.json 2> gpurun_out/fused/legs.err || exit $?
