#!/bin/bash
# Round profile set at the current commit (run through gpurun from the repo root):
# rocprofv3 kernel stats + read/write request counters (tools/profile_gpu.sh) for
# C2, C3 (3 terms + 1 exclude over 1B postings) and C4 (2-4 terms, 4096 queries),
# then the driver's bench command.  Summaries land in gpurun_out/profiles/ (copy
# them into profiles/); PROF_HEAD names the commit (the box has no .git).
#   PROF_HEAD=<commit> bash tools/prof_round.sh <tag-prefix>
set -o pipefail
P=${1:-r03}
ISO="--steps 3 --warmup 1 --no-cpu --latency 0 --inflight 1 --legs none"
export PROF_BASE=/tmp/prof PROF_OUT=gpurun_out/profiles
bash tools/profile_gpu.sh ${P}c2 $ISO && python3 tools/pmc_summary.py ${P}c2 C2 > /dev/null || exit 1
bash tools/profile_gpu.sh ${P}c3 --config C3 --terms 3 --exclude 1 $ISO && python3 tools/pmc_summary.py ${P}c3 C3 > /dev/null || exit 1
bash tools/profile_gpu.sh ${P}c4 --config C3 --nq 4096 --terms 2 --max-terms 4 --qseed 0x59414379000000C7 $ISO && \
  python3 tools/pmc_summary.py ${P}c4 C4 > /dev/null || exit 1
bash tools/fullbench.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/full/bench.json')); print(d['ms_per_step'], {k: v.get('ms_per_step') for k, v in (d.get('legs') or {}).items()})"
