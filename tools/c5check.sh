# GPU: $TESTS first (if set), the whole -m gpu suite, then the headline + C5 legs (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out/c5check
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/c5check/targeted.log 2>&1 || exit $?
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/c5check/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py --legs C5 --no-cpu --latency 0 > gpurun_out/c5check/b.json 2> gpurun_out/c5check/b.err || exit $?
