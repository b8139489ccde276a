# The driver's bench command (--steps 20 --warmup 5, C2 headline only): plain,
# with 300 ms idle before the timed region, and with SDMA copies disabled.
set -o pipefail
mkdir -p gpurun_out/diag
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --legs none --no-cpu --latency 0"
for i in 1 2; do
  timeout -k 10 240 $B > gpurun_out/diag/plain$i.json 2> gpurun_out/diag/plain$i.err || exit $?
  YRWI_BENCH_GAP_MS=300 timeout -k 10 240 $B > gpurun_out/diag/gap$i.json 2> gpurun_out/diag/gap$i.err || exit $?
  HSA_ENABLE_SDMA=0 timeout -k 10 240 $B > gpurun_out/diag/nosdma$i.json 2> gpurun_out/diag/nosdma$i.err || exit $?
done
