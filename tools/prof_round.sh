#!/bin/bash
# Round profile set at the current commit (run through gpurun from the repo root):
# for C2, C3 (3 terms + 1 exclude over 1B postings), C4 (2-4 terms, 4096 queries)
# and C5 custom (authority profile, the 625M-posting shard 0 of 8): rocprofv3
# kernel trace + stats (per-dispatch durations kept), then the read- and
# write-request counter passes, each its own run (tools/profile_gpu.sh), one
# isolated batch in flight.  Summaries in gpurun_out/profiles/ (copy them into
# profiles/); PROF_HEAD names the commit (the box has no .git).
#   PROF_HEAD=<commit> bash tools/prof_round.sh <tag-prefix> [configs]
set -o pipefail
P=${1:-r05}
CFGS=${2:-"C2 C3 C4 C5"}
ISO="--steps 3 --warmup 1 --no-cpu --latency 0 --inflight 1 --legs none"
export PROF_BASE=/tmp/prof PROF_OUT=gpurun_out/profiles
for c in $CFGS; do
  case $c in
    C2) A="" ; name=C2 ;;
    C3) A="--config C3 --terms 3 --exclude 1" ; name=C3 ;;
    C4) A="--config C3 --nq 4096 --terms 2 --max-terms 4 --qseed 0x59414379000000C7" ; name=C4 ;;
    C5) A="--config C5 --shard-of 8 --terms 2 --max-terms 4 --profile custom" ; name=C5_custom ;;
  esac
  t=${P}$(echo $c | tr 'A-Z' 'a-z')
  PROF_T=${PROF_T:-400} bash tools/profile_gpu.sh $t $A $ISO || exit 1
  python3 tools/pmc_summary.py $t $name > /dev/null || exit 1
done
