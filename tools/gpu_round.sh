#!/bin/bash
# One GPU session: GPU parity tests, default bench line, rocprofv3 kernel stats of a bench step.
# Every GPU step has its own time limit.  A step that ends in a fault, abort, segfault or time limit
# (exit 124 / 134 / 137 / 139) ends the script; plain test failures (exit 1) do not stop the bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu ${TEST_ARGS:--x} -v -s --timeout 300 \
    --timeout-method thread ${TEST_SEL:-} > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  echo "tests exit $rc"
  if fatal $rc; then exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?
  echo "bench exit $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate ${PROF_ARGS:-} \
    > gpurun_out/${TAG}_prof_bench.log 2>&1 || exit $?
  cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_kernel_stats.csv
  find gpurun_out/prof -name '*kernel_trace.csv' -delete
fi
