# Why the C5 counter pass fails: one read-request pass, its log kept.
set -o pipefail
mkdir -p gpurun_out/c5pmc
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum \
  --output-format csv -d /tmp/c5pmc -o run -- python3 $R/bench.py --config C5 --shard-of 8 --terms 2 --max-terms 4 \
  --profile custom --steps 3 --warmup 1 --no-cpu --latency 0 --inflight 1 --legs none > $R/gpurun_out/c5pmc/rd.log 2>&1
rc=$?
echo "rc $rc" >> $R/gpurun_out/c5pmc/rd.log
find /tmp/c5pmc -name "*.csv" | head -20 >> $R/gpurun_out/c5pmc/rd.log
exit 0
