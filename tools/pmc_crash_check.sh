# Does rocprofv3 --pmc survive ~200k small kernel dispatches without any yrwi code?
# (round 4's C5 counter pass died with SIGSEGV inside the HIP launch path during the
# index build's 200k per-list launches: profiles/archive/r04_c5_pmc_crash.log.)  Then the same
# pass over libyrwi's C5 index build, untouched (no --kernel-exclude-regex), once.
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/pmccrash
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum --output-format csv -d /tmp/ml -o run \
  -- $R/tools/micro/many_launch 200000 > $R/gpurun_out/pmccrash/many_launch.log 2>&1
echo "many_launch under --pmc: rc=$?" >> $R/gpurun_out/pmccrash/many_launch.log
timeout -s KILL 120 $R/tools/micro/many_launch 200000 > $R/gpurun_out/pmccrash/many_launch_plain.log 2>&1
echo "many_launch plain: rc=$?" >> $R/gpurun_out/pmccrash/many_launch_plain.log
