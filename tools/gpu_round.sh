#!/bin/bash
# One GPU session: GPU parity tests, default bench line, rocprofv3 kernel stats of a bench step.
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
if [ "${SKIP_PROF:-0}" != "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.log 2>&1
  cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_kernel_stats.csv
  find gpurun_out/prof -name '*kernel_trace.csv' -delete
fi
