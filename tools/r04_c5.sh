# Kernel stats of the C5 custom (authority) leg and of C3 with the fused chain.
set -o pipefail
mkdir -p gpurun_out/kst
KARGS="--config C5 --shard-of 8 --terms 2 --max-terms 4 --profile custom" bash tools/kstats.sh c5c || exit 1
KARGS="--config C3 --terms 3 --exclude 1" bash tools/kstats.sh c3fused || exit 1
mv gpurun_out/c5c_kstats.txt gpurun_out/c3fused_kstats.txt gpurun_out/kst/
