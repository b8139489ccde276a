# Round-4 validation: the -m gpu suite (per-test lines), smoke, then the headline
# bench (C2, legs none, CPU baseline + parity from the timed buffers); every step
# under its own time limit, stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/val
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/val/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --legs none \
  > gpurun_out/val/c2.json 2> gpurun_out/val/c2.err || exit $?
