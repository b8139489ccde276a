set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards_loopback.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/tp -o run -- python3 $R/tools/tailprobe.py > $R/gpurun_out/tp.log 2>&1
python3 - > $R/gpurun_out/tp.txt <<'PY'
import sys; sys.path.insert(0, "/root/repo/tools")
from kstats_summary import dispatches
for k in ("k_shard_fin", "k_reduce", "k_compact", "k_join", "k_probe(", "k_score(", "k_topq", "k_emit", "k_partition"):
    print(k, " ".join("%.0f" % d for d in dispatches("/tmp/tp", k)))
PY
