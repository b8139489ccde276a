# Host counts: GPU suite, the phase counters for C5 custom (profiling build), C5 kernel stats and legs.
set -o pipefail
mkdir -p gpurun_out/hc gpurun_out/kst
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/hc/t.log 2>&1 || exit $?
CP_MAX_TERMS=4 YRWI_LIB=$PWD/yacy_search_server_amd/libyrwi_cprof.so timeout -k 10 400 python3 -u tools/chain_prof.py C5 2 0 custom 8 \
  > gpurun_out/hc/c5.json 2> gpurun_out/hc/c5.err || exit $?
KARGS="--config C5 --shard-of 8 --terms 2 --max-terms 4 --profile custom" bash tools/kstats.sh c5hc2 || exit 1
mv gpurun_out/c5hc2_kstats.txt gpurun_out/kst/
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C5,C3 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/hc/legs.json 2> gpurun_out/hc/legs.err || exit $?
