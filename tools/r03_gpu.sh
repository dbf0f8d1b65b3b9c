#!/bin/bash
# Round-3 GPU session helper: each step under its own time limit; a fault / abort / segfault / time
# limit (124 / 134 / 137 / 139) ends the script, plain test failures (1) do not.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ "${ISA:-0}" = "1" ]; then
  timeout -k 10 120 ./tools/isa_rate > gpurun_out/${TAG}_isa_rate.log 2>&1
  rc=$?; echo "isa_rate exit $rc"; if fatal $rc; then exit $rc; fi
fi
if [ -n "${AB:-}" ]; then  # AB="--env X --values a,b ..." : tools/conv_ab.py
  timeout -k 10 ${AB_TIMEOUT:-300} python -u tools/conv_ab.py ${AB} > gpurun_out/${TAG}_conv_ab.log 2>&1
  rc=$?; echo "conv_ab exit $rc"; if fatal $rc; then exit $rc; fi
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${TESTS} -m gpu ${TESTK:+-k "$TESTK"} \
    --maxfail=${MAXFAIL:-10} -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?; echo "tests exit $rc"; if fatal $rc; then exit $rc; fi
fi
if [ "${SENS:-0}" = "1" ]; then
  timeout -k 10 300 python -u tools/depth_sensitivity.py > gpurun_out/${TAG}_depth_sens.log 2>&1
  rc=$?; echo "sens exit $rc"; if fatal $rc; then exit $rc; fi
  RDMI_DEPTH_F32=0 timeout -k 10 300 python -u tools/depth_sensitivity.py > gpurun_out/${TAG}_depth_sens_f16.log 2>&1
  rc=$?; echo "sens f16 exit $rc"; if fatal $rc; then exit $rc; fi
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?; echo "bench exit $rc"; if fatal $rc; then exit $rc; fi
fi
if [ "${PMC:-0}" = "1" ]; then
  OUT=gpurun_out/${TAG}_pmc PRESET=${PMC_PRESET:-fast} bash tools/pmc_bench.sh > gpurun_out/${TAG}_pmc.log 2>&1
  rc=$?; echo "pmc exit $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${PROF:-0}" = "1" ]; then
  rm -rf gpurun_out/${TAG}_prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate ${PROF_ARGS:-} \
    > gpurun_out/${TAG}_prof_bench.log 2>&1
  rc=$?; echo "prof exit $rc"; if fatal $rc; then exit $rc; fi
  cp "$(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_kernel_stats.csv
  find gpurun_out/${TAG}_prof -name '*kernel_trace.csv' -delete
fi
exit 0
