#!/bin/bash
# A/B of whole trees on one box: bench.py's legs (LEGS, default C5) with the
# in-tree build and with the tree under each DIR (a checkout of another commit,
# built), alternating, twice.  One JSON line per run in gpurun_out/legab/.
set -o pipefail
mkdir -p gpurun_out/legab
LEGS=${LEGS:-C5}
ARGS=${LEG_ARGS:-"--steps 5 --warmup 2 --no-cpu --latency 0 --check 0 --leg-check 4 --leg-latency 0"}
root=$(pwd)
for i in 1 2; do
  for d in cur $DIRS; do
    n=$(basename $d)
    if [ "$d" = cur ]; then cd "$root"; else cd "$root/$d"; fi
    timeout -k 10 300 python3 -u bench.py $ARGS --legs $LEGS > "$root/gpurun_out/legab/${n}_$i.json" \
      2> "$root/gpurun_out/legab/${n}_$i.err" || exit $?
    cd "$root"
    python3 -c "
import json; d=json.loads(open('gpurun_out/legab/${n}_$i.json').read().strip().splitlines()[-1])
print('$n', $i, round(d['ms_per_step'],4), {k: round(v['ms_per_step'],4) for k, v in d['legs'].items()})"
  done
done
