# GPU occupancy of the headline's timed region (rocprofv3 kernel trace; 50 ms idle
# gaps bracket the region): tools/busy_union.py on the box -> gpurun_out/busy/.
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/busy
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/busy
YRWI_BENCH_GAP_MS=50 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/busy -o run -- \
  python3 $R/bench.py --steps 40 --warmup 8 --no-cpu --latency 0 --legs none $BARGS > $R/gpurun_out/busy/b.log 2>&1 || exit $?
f=$(find /tmp/busy -name "*kernel_trace.csv" | head -1)
python3 $R/tools/busy_union.py $f 50 > $R/gpurun_out/busy/union.txt 2>&1
cat $R/gpurun_out/busy/union.txt
