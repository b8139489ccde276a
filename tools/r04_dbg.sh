set -o pipefail
mkdir -p gpurun_out/dbg
YRWI_SYNC_DEBUG=1 timeout -k 10 100 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 90 --timeout-method thread \
  -k "forced_join and tiny" > gpurun_out/dbg/t.log 2>&1
