# Round check at HEAD (run through gpurun from the repo root): the whole GPU suite,
# then the driver's bench command.  Output in gpurun_out/final/.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/final/t.log 2>&1 || exit $?
timeout -k 10 1000 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/b.json 2> gpurun_out/final/b.err || exit $?
