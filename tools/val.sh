# GPU validation: the -m gpu suite, smoke, then the driver's bench command twice
# (C2 headline only) -- every step under its own time limit, stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/val
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/val/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val/smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --legs none --no-cpu --latency 0 \
    > gpurun_out/val/drv$i.json 2> gpurun_out/val/drv$i.err || exit $?
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --legs none --no-cpu \
  > gpurun_out/val/long.json 2> gpurun_out/val/long.err || exit $?
