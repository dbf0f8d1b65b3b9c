# Round-3 session-2 final GPU batch: full GPU tests, smoke, default bench, kernel-stats profile of a bench step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/hb.sh timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=20 --timeout 300 --timeout-method thread > gpurun_out/r03s_gpu_tests.log 2>&1; rc=$?
echo "tests exit $rc"
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/hb.sh timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s_smoke.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r03s_bench.log 2>&1 || exit $?
rm -rf gpurun_out/r03s_prof
bash tools/hb.sh timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate > gpurun_out/r03s_prof_bench.log 2>&1 || exit $?
cp "$(find gpurun_out/r03s_prof -name '*kernel_stats.csv' | head -1)" gpurun_out/r03s_kernel_stats.csv
find gpurun_out/r03s_prof -name '*kernel_trace.csv' -delete
