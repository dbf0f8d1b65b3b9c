# round 6 final validation after the GroupNorm-transform priority default (session q): full GPU test suite, smoke, default bench line, rocprofv3 kernel stats,
# per-shape table of one step.  Every GPU step under its own limit; a fault / abort / time limit ends it.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash tools/hb.sh timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 \
  --timeout-method thread > gpurun_out/r06zz_gpu_tests.log 2>&1; rc=$?; echo "tests exit $rc"; fatal $rc && exit $rc
bash tools/hb.sh timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zz_smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; fatal $rc && exit $rc
bash tools/hb.sh timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r06zz_bench.log 2>&1
rc=$?; echo "bench exit $rc"; fatal $rc && exit $rc
rm -rf gpurun_out/prof
bash tools/hb.sh timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate > gpurun_out/r06zz_prof_bench.log 2>&1
rc=$?; echo "prof exit $rc"; fatal $rc && exit $rc
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/r06zz_kernel_stats.csv
find gpurun_out/prof -name '*kernel_trace.csv' -delete
RDMI_PROF_SHAPES=1 bash tools/hb.sh timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline \
  --no-validate > gpurun_out/r06zz_shapes.log 2>&1; echo "shapes exit $?"
