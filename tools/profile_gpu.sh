#!/bin/bash
# Profile bench.py on the GPU box with rocprofv3 (run through gpurun from the repo root).
#   pass 1: --kernel-trace --stats                              -> per-kernel durations
#   pass 2: --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum + _DRAM_sum    -> read requests leaving L2, by size
#   pass 3: --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum         -> write requests (64 B, the rest 32 B)
# Each counter pass is its own run (MI355X_MICROARCH.md, HBM / rocprofv3).  Request
# sizes are counted exactly, so no FETCH_SIZE correction is needed: on this path the
# reads are 128-B requests (gathers and streams alike).  Raw rocprofv3 output goes
# to /tmp/prof/<tag>/ on the box (it is far larger than what gpurun copies back);
# tools/pmc_summary.py, run right after on the box with PROF_BASE=/tmp/prof and
# PROF_OUT=gpurun_out/profiles, writes the summaries that are kept.
set -e
TAG=${1:-r02}
shift || true
ARGS=${@:---steps 5 --warmup 2 --no-cpu --latency 0 --inflight 1 --legs none}
ROOT=$(pwd)
OUT=/tmp/prof/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
echo "[$TAG] kernel trace" >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $ROOT/bench.py $ARGS > $OUT/kt.log 2>&1
# counters only for the query path: the index build's per-list launches (C5: 100k
# lists, 200k dispatches) crashed rocprofv3's counter collection (SIGSEGV in
# launch_features, gpurun_out/c5pmc/rd.log of round 4)
EXCL=${PROF_EXCL:-"k_validate|k_features|rocprim|k_dict|k_uid|k_bitmap|k_heads|k_pad|k_gather"}
echo "[$TAG] read requests" >&2
timeout -s KILL ${PROF_T:-200} rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum --kernel-exclude-regex "$EXCL" --output-format csv -d $OUT/rd -o run -- python3 $ROOT/bench.py $ARGS > $OUT/rd.log 2>&1
echo "[$TAG] write requests" >&2
timeout -s KILL ${PROF_T:-200} rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-exclude-regex "$EXCL" --output-format csv -d $OUT/wr -o run -- python3 $ROOT/bench.py $ARGS > $OUT/wr.log 2>&1
echo done
