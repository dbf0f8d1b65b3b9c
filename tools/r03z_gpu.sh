# Final build: HBM traffic passes (FETCH_SIZE / WRITE_SIZE) and rocprofv3 kernel stats of a bench step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r03z_pmc gpurun_out/r03z_prof
OUT=gpurun_out/r03z_pmc PMC_TIMEOUT=300 bash tools/hb.sh bash tools/pmc_bench.sh > gpurun_out/r03z_pmc.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03z_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate > gpurun_out/r03z_prof_bench.log 2>&1 || exit $?
cp "$(find gpurun_out/r03z_prof -name '*kernel_stats.csv' | head -1)" gpurun_out/r03z_kernel_stats.csv
find gpurun_out/r03z_prof -name '*kernel_trace.csv' -delete
