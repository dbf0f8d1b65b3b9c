#!/bin/bash
# One parametrised GPU session (replaces the per-experiment r03*_gpu.sh one-offs).
#
#   TAG=r04a STEPS="tests smoke bench shapes prof" bash tools/gpu_run.sh
#
# Steps, run in the order given, each under its own time limit, output in gpurun_out/${TAG}_<step>.*:
#   tests    pytest -m gpu (TEST_K: a -k expression, TEST_SEL: test paths, TEST_ARGS: more options)
#   smoke    __graft_entry__.smoke()
#   bench    bench.py ${BENCH_ARGS} (default preset, --steps ${BENCH_STEPS:-3} --warmup 2)
#   shapes   one step with RDMI_PROF_SHAPES=1 (per-launch-shape TF/s table in the JSON line)
#   prof     rocprofv3 --kernel-trace --stats of one bench step → ${TAG}_kernel_stats.csv
#   pmc      FETCH_SIZE / WRITE_SIZE passes of one bench step → ${TAG}_pmc/ (tools/pmc_bench.sh)
#   kbench   python tools/kbench.py ${KBENCH_ARGS}
#   cmd      an arbitrary command: CMD="python -u tools/x.py" (its own limit CMD_TIMEOUT, default 300)
# Exit codes 124 / 134 / 137 / 139 (time limit, abort, kill, segfault) end the session at once; a plain
# test failure (exit 1) does not stop the later steps.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
STEPS=${STEPS:-"tests smoke bench"}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
hb() { bash tools/hb.sh "$@"; }
for s in $STEPS; do
  case $s in
    tests)
      hb timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TEST_SEL:-tests} -m gpu -q ${TEST_ARGS:---maxfail=20} \
        --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$? ;;
    smoke)
      hb timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$? ;;
    bench)
      hb timeout -k 10 ${BENCH_TIMEOUT:-500} python -u bench.py --steps ${BENCH_STEPS:-3} --warmup 2 ${BENCH_ARGS:-} \
        > gpurun_out/${TAG}_bench.log 2>&1; rc=$? ;;
    shapes)
      RDMI_PROF_SHAPES=1 hb timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate \
        ${BENCH_ARGS:-} > gpurun_out/${TAG}_shapes.log 2>&1; rc=$? ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-validate ${BENCH_ARGS:-} \
        > gpurun_out/${TAG}_prof_bench.log 2>&1; rc=$?
      if [ $rc -eq 0 ]; then
        cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/${TAG}_kernel_stats.csv
        find gpurun_out/prof -name '*kernel_trace.csv' -delete
      fi ;;
    pmc)
      OUT=gpurun_out/${TAG}_pmc bash tools/pmc_bench.sh > gpurun_out/${TAG}_pmc.log 2>&1; rc=$? ;;
    kbench)
      hb timeout -k 10 ${KBENCH_TIMEOUT:-400} python -u tools/kbench.py ${KBENCH_ARGS:-} > gpurun_out/${TAG}_kbench.log 2>&1; rc=$? ;;
    cmd)
      hb timeout -k 10 ${CMD_TIMEOUT:-300} $CMD > gpurun_out/${TAG}_cmd.log 2>&1; rc=$? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "$s exit $rc"
  if fatal $rc; then exit $rc; fi
done
