#!/bin/bash
# Profile bench.py on the GPU box with rocprofv3 (run through gpurun from the repo root).
#   pass 1: --kernel-trace --stats          -> per-kernel durations
#   pass 2: --pmc FETCH_SIZE  (own pass)    -> HBM read bytes (x2 on gfx950, MI355X_MICROARCH.md §HBM)
#   pass 3: --pmc WRITE_SIZE  (own pass)    -> HBM write bytes
# Outputs under gpurun_out/prof/<tag>/ ; tools/pmc_summary.py turns them into profiles/*.
set -e
TAG=${1:-r01}
shift || true
ARGS=${@:---steps 5 --warmup 2 --no-cpu --latency 0 --inflight 1 --legs none}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $ROOT/bench.py $ARGS > $OUT/kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ROOT/bench.py $ARGS > $OUT/write.log 2>&1
echo done
