set -e
mkdir -p gpurun_out/cfg gpurun_out/prof
timeout -k 10 200 python -u bench.py > gpurun_out/cfg/C2_default.json 2> gpurun_out/cfg/C2_default.err
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --latency 0 > gpurun_out/cfg/C2_s5w1.json 2> gpurun_out/cfg/C2_s5w1.err
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --latency 20 --config C5 --shard-of 8 --terms 2 --max-terms 4 --profile custom --cpu-budget 6 > gpurun_out/cfg/C5.json 2> gpurun_out/cfg/C5.err
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/c3 -o run -- python3 $R/bench.py --config C3 --terms 3 --exclude 1 --steps 2 --warmup 1 --no-cpu --latency 0 --inflight 1 > $R/gpurun_out/prof/c3.log 2>&1
