set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1
bash tools/kstats.sh b
timeout -k 10 200 python bench.py --no-cpu --latency 0 > gpurun_out/bench_j.json 2>gpurun_out/bench.err
