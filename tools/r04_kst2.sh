# Kernel stats: C5 custom (k_hostcount + k_reduce) and C3 with the fused chain.
set -o pipefail
mkdir -p gpurun_out/kst
KARGS="--config C5 --shard-of 8 --terms 2 --max-terms 4 --profile custom" bash tools/kstats.sh c5hc || exit 1
KARGS="--config C3 --terms 3 --exclude 1" bash tools/kstats.sh c3lds || exit 1
mv gpurun_out/c5hc_kstats.txt gpurun_out/c3lds_kstats.txt gpurun_out/kst/
