set -e
mkdir -p gpurun_out/var
for i in 1 2 3; do
timeout -k 10 200 python -u bench.py --no-cpu --latency 0 > gpurun_out/var/b$i.json 2> gpurun_out/var/b$i.err
done
timeout -k 10 200 python -u bench.py --no-cpu --latency 0 --inflight 3 > gpurun_out/var/b_if3.json 2> gpurun_out/var/b_if3.err
YRWI_LANES=3 timeout -k 10 200 python -u bench.py --no-cpu --latency 0 --inflight 3 > gpurun_out/var/b_l3.json 2> gpurun_out/var/b_l3.err
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/var/kt -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --latency 0 > $R/gpurun_out/var/kt.log 2>&1
