# HBM traffic of one fast-preset step on the final round-3 build (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r03t_pmc
OUT=gpurun_out/r03t_pmc PMC_TIMEOUT=300 bash tools/hb.sh bash tools/pmc_bench.sh > gpurun_out/r03t_pmc.log 2>&1 || exit $?
