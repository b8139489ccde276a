# Round-5 diagnosis: (1) the stale HIP error after authority queries (AMD_LOG_LEVEL=1
# names the failing API call); (2) k_compact cost attribution on C2 (YRWI_COMPACT_WHATIF
# builds); (3) does rocprofv3 --pmc survive 200k small dispatches (no yrwi code)?
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/diag1
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/diag1/incr.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
bash tools/kvar.sh cur=cur w1=gpurun_var/libyrwi_w1.so w2=gpurun_var/libyrwi_w2.so w3=gpurun_var/libyrwi_w3.so \
  w4=gpurun_var/libyrwi_w4.so > gpurun_out/diag1/kvar.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum --output-format csv -d /tmp/ml -o run \
  -- $R/tools/micro/many_launch 200000 > $R/gpurun_out/diag1/many_launch_pmc.log 2>&1
echo "many_launch rc=$?" >> $R/gpurun_out/diag1/many_launch_pmc.log
