# GPU check of a change (run through gpurun from the repo root): the tests named in
# $TESTS first (default: none), then the whole -m gpu suite, then (BENCH=1) the
# driver's bench command.  Every step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/check
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/check/targeted.log 2>&1 || exit $?
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/check/gpu_tests.log 2>&1 || exit $?
if [ "$BENCH" = "1" ]; then
  timeout -k 10 1000 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/check/b.json 2> gpurun_out/check/b.err || exit $?
fi
