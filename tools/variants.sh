#!/bin/bash
# Kernel-variant sweep on the GPU box: for each gpurun_var/libyrwi_*.so (plus the
# in-tree build) one bench line and the per-kernel average durations.
set -e
R=$(pwd)
mkdir -p $R/gpurun_out/var
cd /tmp && export TMPDIR=/tmp
for L in $R/yacy_search_server_amd/libyrwi.so $R/gpurun_var/libyrwi_*.so; do
  n=$(basename $L .so)
  YRWI_LIB=$L timeout -k 10 200 python3 $R/bench.py --cpu-budget 1 --latency 0 > $R/gpurun_out/var/$n.json 2> $R/gpurun_out/var/$n.err
  rm -rf /tmp/kv
  YRWI_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kv -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --latency 0 --inflight 1 > /tmp/kv.log 2>&1
  python3 - $n $R/gpurun_out/var/$n.json <<'PY' >> $R/gpurun_out/var/summary.txt
import csv, glob, json, sys
f = glob.glob("/tmp/kv/**/*kernel_stats.csv", recursive=True)[0]
k = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step %.3f" % b["ms_per_step"], "mismatch %s" % (b.get("parity_sample") or {}).get("mismatches"), " ".join("%s %.1f" % (n.split("::")[-1], v) for n, v in k.items() if n.split("::")[-1] in ("k_compact", "k_join", "k_score", "k_probe", "k_partition", "k_score_full")))
PY
done
cat $R/gpurun_out/var/summary.txt
