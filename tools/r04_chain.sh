# Chained folds: the whole GPU suite, the C3 / C4 / C5 legs of the bench, C3 kernel
# stats and the host-side breakdown of C4 batches.
set -o pipefail
mkdir -p gpurun_out/chain gpurun_out/kst gpurun_out/c4p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/chain/t1.log 2>&1 || exit $?
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4,C5 --latency 0 --leg-latency 0 \
  --no-cpu > gpurun_out/chain/legs.json 2> gpurun_out/chain/legs.err || exit $?
KARGS="--config C3 --terms 3 --exclude 1" bash tools/kstats.sh c3grp || exit 1
mv gpurun_out/c3grp_kstats.txt gpurun_out/kst/
YRWI_HOST_PROF=1 timeout -k 10 300 python3 -u bench.py --config C3 --nq 4096 --terms 2 --max-terms 4 --steps 4 --warmup 2 \
  --no-cpu --latency 0 --legs none --batches 2 --check 2 --inflight 2 > gpurun_out/c4p/b.json 2> gpurun_out/c4p/b.err || exit $?
