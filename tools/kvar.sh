#!/bin/bash
# Kernel stats of library variants: for each NAME=LIB[:ENV=VAL] one isolated
# rocprofv3 kernel-stats run (tools/kstats.sh) and the headline bench line.
#   bash tools/kvar.sh cur=cur base=cur:YRWI_BAND_ORDER=0 ct2=gpurun_var/libyrwi_ct2.so
# KARGS: extra bench.py arguments for both runs (e.g. the C3 workload)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/kvar
for nv in "$@"; do
  n=${nv%%=*}; rest=${nv#*=}; p=${rest%%:*}; e=""
  [ "$rest" != "$p" ] && e=${rest#*:}
  ( if [ "$p" = cur ]; then unset YRWI_LIB; else export YRWI_LIB=$R/$p; fi
    [ -n "$e" ] && export "$e"
    bash tools/kstats.sh kv_$n || exit 1
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 16 --no-cpu --latency 0 --legs none $KARGS > gpurun_out/kvar/$n.json 2> gpurun_out/kvar/$n.err || exit 1
  ) || exit 1
  mv gpurun_out/kv_${n}_kstats.txt gpurun_out/kvar/
  python3 - $n <<'PY'
import json, sys
n = sys.argv[1]
k, c = {}, {}
for l in open(f"gpurun_out/kvar/kv_{n}_kstats.txt"):
    f = l.split()
    if len(f) >= 4:  # template instances (k_probe<true> / <false>) pool: mean per dispatch
        name = " ".join(f[:-3]).split("::")[-1].split("<")[0]
        k[name] = k.get(name, 0.0) + float(f[-2]) * int(f[-3])
        c[name] = c.get(name, 0) + int(f[-3])
k = {x: k[x] / c[x] for x in k if c[x]}
d = json.load(open(f"gpurun_out/kvar/{n}.json"))
print(n, "ms/step %.4f" % d["ms_per_step"], " ".join("%s %.1f" % (x, k.get(x, 0)) for x in ("k_compact", "k_probe", "k_tile_order", "k_join", "k_score", "k_reduce")))
PY
done
