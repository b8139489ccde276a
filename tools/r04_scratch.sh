# C4 with larger per-lane scratch budgets (fewer passes per batch), host breakdown kept.
set -o pipefail
mkdir -p gpurun_out/scr
for gb in 24 32; do
  YRWI_SCRATCH_GB=$gb timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C4 --latency 0 \
    --leg-latency 0 --no-cpu > gpurun_out/scr/legs_$gb.json 2> gpurun_out/scr/legs_$gb.err || exit $?
done
