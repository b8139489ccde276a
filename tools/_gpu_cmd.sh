set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c5 or authority or bit_exact or loopback or java or nodes or filters" > gpurun_out/gpu_tests.log 2>&1 && \
bash tools/kstats_cfg.sh c5c --config C5 --shard-of 8 --profile custom --terms 2 --max-terms 4 --steps 5 --warmup 2
