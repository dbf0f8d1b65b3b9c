#!/bin/bash
# scratch: GEMM shapes
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kbench.py --only gemm || exit 1
