# The driver's bench command at HEAD (one MI355X), its JSON line and log kept.
set -o pipefail
mkdir -p gpurun_out/bench
timeout -k 10 1100 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench/b.json 2> gpurun_out/bench/b.err || exit $?
