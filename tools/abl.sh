#!/bin/bash
# scratch A/B: halo conv variants with the fused input GroupNorm (RDMI_CONV_HALO 2 = default, 3 = two workgroups per CU everywhere)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for h in 2 3; do
  echo "== RDMI_CONV_HALO=$h"
  RDMI_CONV_HALO=$h timeout -k 10 200 python -u tools/kbench.py --only gnconv || exit 1
done
