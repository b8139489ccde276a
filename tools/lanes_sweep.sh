#!/bin/bash
# Lanes / batches-in-flight sweep on the GPU box (3 bench runs each, ms per step).
set -e
R=$(pwd)
mkdir -p $R/gpurun_out/lanes
for L in 2 3 4; do
  for i in 1 2 3; do
    YRWI_LANES=$L timeout -k 10 200 python3 $R/bench.py --no-cpu --latency 0 --inflight $L > $R/gpurun_out/lanes/l${L}_$i.json 2> $R/gpurun_out/lanes/l${L}_$i.err
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lanes', sys.argv[2], 'ms/step %.3f' % b['ms_per_step'])" $R/gpurun_out/lanes/l${L}_$i.json $L >> $R/gpurun_out/lanes/summary.txt
  done
done
cat $R/gpurun_out/lanes/summary.txt
