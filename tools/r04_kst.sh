# Kernel stats of one isolated batch for C3 and C4 (rocprofv3 kernel trace), chain on and off.
set -o pipefail
mkdir -p gpurun_out/kst
KARGS="--config C3 --terms 3 --exclude 1" bash tools/kstats.sh c3on || exit 1
YRWI_NO_CHAIN=1 KARGS="--config C3 --terms 3 --exclude 1" bash tools/kstats.sh c3off || exit 1
mv gpurun_out/c3on_kstats.txt gpurun_out/c3off_kstats.txt gpurun_out/kst/
