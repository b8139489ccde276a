# The driver's round-end bench command exactly (default legs, CPU baseline), under a time limit.
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || exit $?
