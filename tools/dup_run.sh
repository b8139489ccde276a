set -o pipefail
mkdir -p gpurun_out/t2
timeout -k 10 300 python -u -m pytest tests/test_java_sequence.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2/t.log 2>&1 || exit $?
AB_ARGS="--steps 40 --warmup 8 --no-cpu --latency 0 --legs none" bash tools/ab.sh base=cur compact=gpurun_var/libyrwi_dup_compact.so probe=gpurun_var/libyrwi_dup_probe.so reduce=gpurun_var/libyrwi_dup_reduce.so shardfin=gpurun_var/libyrwi_dup_shardfin.so combine=gpurun_var/libyrwi_dup_combine.so emit=gpurun_var/libyrwi_dup_emit.so copyin=gpurun_var/libyrwi_dup_copyin.so qtabs=gpurun_var/libyrwi_dup_qtabs.so topq=gpurun_var/libyrwi_dup_topq.so
