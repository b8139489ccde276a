# Host counts read before compare-and-swap: rank-phase GPU tests, C5 kernel stats and legs.
set -o pipefail
mkdir -p gpurun_out/c5b gpurun_out/kst
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/c5b/t.log 2>&1 || exit $?
KARGS="--config C5 --shard-of 8 --terms 2 --max-terms 4 --profile custom" bash tools/kstats.sh c5b || exit 1
mv gpurun_out/c5b_kstats.txt gpurun_out/kst/
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C5 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/c5b/legs.json 2> gpurun_out/c5b/legs.err || exit $?
