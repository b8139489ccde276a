set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "forced_join or bit_exact" > gpurun_out/gputest.log 2>&1
for r in 16 32 64; do YRWI_PROBE_RATIO=$r timeout -k 10 200 python bench.py --no-cpu --latency 0 > gpurun_out/bench_r$r.json 2>/dev/null; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/hip -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --latency 0 > $GRAFT_REPO_ROOT/gpurun_out/hip.log 2>&1
