#!/bin/bash
# Band-major tile schedule A/B: GPU suite, kernel stats with the band order on
# and off, and the driver's bench command with each (YRWI_BAND_ORDER=0/1).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/band
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/band/gpu_tests.log 2>&1 || { tail -30 gpurun_out/band/gpu_tests.log; exit 1; }
tail -2 gpurun_out/band/gpu_tests.log
for b in 1 0; do
  YRWI_BAND_ORDER=$b bash tools/kstats.sh band$b || exit 1
  mv gpurun_out/band${b}_kstats.txt gpurun_out/band/ 
  head -12 gpurun_out/band/band${b}_kstats.txt
done
for i in 1 2; do for b in 1 0; do
  YRWI_BAND_ORDER=$b timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --latency 0 --legs none > gpurun_out/band/bench_b${b}_$i.json 2> gpurun_out/band/bench_b${b}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/band/bench_b${b}_$i.json')); print('band', $b, $i, round(d['ms_per_step'],4), d.get('roofline',{}).get('frac'))"
done; done
