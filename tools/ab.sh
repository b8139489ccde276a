#!/bin/bash
# A/B of library builds on one box: bench.py (no CPU leg) with each YRWI_LIB in turn,
# twice, one JSON line per run into gpurun_out/ab/<name>_<i>.json.
#   bash tools/ab.sh name1=path1.so name2=path2.so ...   (path "cur" = the in-tree build)
set -e
mkdir -p gpurun_out/ab
ARGS=${AB_ARGS:---steps 20 --warmup 5 --no-cpu --latency 0}
for i in $(seq 1 ${ROUNDS:-2}); do
  for nv in "$@"; do
    n=${nv%%=*}; p=${nv#*=}
    if [ "$p" = cur ]; then unset YRWI_LIB; else export YRWI_LIB=$(pwd)/$p; fi
    timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/ab/${n}_$i.json 2> gpurun_out/ab/${n}_$i.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${n}_$i.json')); print('$n', $i, round(d['ms_per_step'],4), d['phase_ms'])"
  done
done
