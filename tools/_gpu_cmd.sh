set -e

R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst -o run -- python3 $R/tools/bench_rows.py > $R/gpurun_out/kst.log 2>&1
python3 $R/tools/kstats_summary.py /tmp/kst $R/gpurun_out/rows_kstats.txt k_event_add
