# k_compact tiles-per-workgroup / matches-per-thread on the chained-fold legs (C3, C4):
# the head build, four variant builds (yacy_search_server_amd/var/), the head build again.
set -o pipefail
D=gpurun_out/csweep${TAG:-}
mkdir -p $D
for v in ${SWEEP:-head t2 t8 u2 u8 head2}; do
  case $v in head*) L=$PWD/yacy_search_server_amd/libyrwi.so ;; *) L=$PWD/yacy_search_server_amd/var/libyrwi_$v.so ;; esac
  YRWI_LIB=$L timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs C3,C4 --latency 0 \
    --leg-latency 0 --no-cpu > $D/$v.json 2> $D/$v.err || exit $?
  echo "$v done"
done
