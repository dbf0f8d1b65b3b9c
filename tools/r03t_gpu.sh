# HBM traffic of one fast-preset step on the final round-3 build (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r03t_pmc
OUT=gpurun_out/r03t_pmc PMC_TIMEOUT=300 bash tools/hb.sh bash tools/pmc_bench.sh > gpurun_out/r03t_pmc.log 2>&1 || exit $?
# multi-rank rehearsal on the final build: 2 ranks sharing the one GPU over gloo (not a scaling number)
RDMI_BENCH_SHARED_GPU=1 bash tools/hb.sh timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --frames-total 30 --no-cpu-baseline > gpurun_out/r03t_shared2.log 2>&1 || exit $?
