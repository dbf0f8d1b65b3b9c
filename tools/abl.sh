#!/bin/bash
# scratch A/B: fused GroupNorm conv, wave priority of the normalising segment
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for pr in 0 1 2 3; do
  echo "== RDMI_GN_PRIO=$pr"
  RDMI_GN_PRIO=$pr timeout -k 10 200 python -u tools/kbench.py --only gnconv || exit 1
done
