#!/bin/bash
# scratch A/B: small-K GEMM engine (RDMI_GEMM_OCC2 0 = off, 1 = K <= 640, 2 = every dense GEMM)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in 0 2; do
  echo "== RDMI_GEMM_OCC2=$o"
  RDMI_GEMM_OCC2=$o timeout -k 10 200 python -u tools/kbench.py --only gemm || exit 1
done
