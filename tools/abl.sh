#!/bin/bash
# scratch A/B: attention wave priority (RDMI_ATTN_PRIO 0 = flips around MFMA blocks, 1 = none, 2 = static for waves 4-7)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for pr in 0 1 2 0; do
  echo "== RDMI_ATTN_PRIO=$pr"
  RDMI_ATTN_PRIO=$pr timeout -k 10 200 python -u tools/kbench.py --only attn || exit 1
done
