# Targeted GPU tests of the working tree, then an A/B of library builds (tools/ab.sh)
# and the in-tree build's kernel stats.  AB: "name=path ..." pairs (path "cur" = in tree).
set -o pipefail
mkdir -p gpurun_out/abr
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/abr/tests.log 2>&1 || exit $?
fi
AB_ARGS=${AB_ARGS:-"--steps 40 --warmup 8 --no-cpu --latency 0 --legs none"} bash tools/ab.sh $AB || exit $?
if [ -n "$KSTATS" ]; then  # every build's isolated kernel times, same box
  for nv in $AB; do
    n=${nv%%=*}; p=${nv#*=}
    if [ "$p" = cur ]; then unset YRWI_LIB; else export YRWI_LIB=$(pwd)/$p; fi
    bash tools/kstats.sh abr_$n || exit $?
  done
fi
