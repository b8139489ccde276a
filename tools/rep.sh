#!/bin/bash
# Repeat the headline bench (no legs, no CPU leg) to see run-to-run spread:
#   bash tools/rep.sh <reps> [extra bench args]
set -e
N=$1; shift
mkdir -p gpurun_out/rep
for i in $(seq 1 $N); do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 6 --no-cpu --latency 0 --legs none "$@" > gpurun_out/rep/$i.json 2> gpurun_out/rep/$i.err
  python3 -c "import json; d=json.load(open('gpurun_out/rep/$i.json')); print($i, round(d['ms_per_step'],4), d['phase_ms']['host_total'])"
done
