# Host-side breakdown of C4 batches (4096 x 2-4 terms over the C3 corpus): passes, plan, join, rank.
set -o pipefail
mkdir -p gpurun_out/c4p
YRWI_HOST_PROF=1 timeout -k 10 400 python3 -u bench.py --config C3 --nq 4096 --terms 2 --max-terms 4 --steps 4 --warmup 2 \
  --no-cpu --latency 0 --legs none --batches 2 --check 2 --inflight 2 > gpurun_out/c4p/b.json 2> gpurun_out/c4p/b.err || exit $?
