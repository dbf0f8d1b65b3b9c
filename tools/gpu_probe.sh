#!/bin/bash
# One GPU session: kernel tests, engine A/B microbenchmarks, host-overhead probe, kernel trace of
# one bench step (idle-gap analysis).  Every GPU step has its own time limit; stop at first failure.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/p_tests.log 2>&1
RDMI_GEMM_PP=0 timeout -k 10 200 python tools/kbench.py --only conv > gpurun_out/p_kb_classic.log 2>&1
timeout -k 10 300 python tools/kbench.py --only conv,gemm,gn > gpurun_out/p_kb_pp.log 2>&1
if [ "${PROBE_TRACE:-1}" = "1" ]; then
  rm -rf gpurun_out/trace
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/p_trace_bench.log 2>&1
  python3 tools/gaps.py "$(find gpurun_out/trace -name '*kernel_trace.csv' | head -1)" > gpurun_out/p_gaps.log 2>&1
  find gpurun_out/trace -name '*kernel_trace.csv' -delete
fi
