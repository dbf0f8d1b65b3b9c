#!/bin/bash
# Segment breakdown of conv_halo_occ2_kernel over epilogue variants (tools/conv_stamp.hip; build it first):
#   bash tools/conv_stamp_sweep.sh ["B HW gn res mom Cin Cout rstride" ...]
# Default: the 768² 128 → 128 GroupNorm-input conv with each of residual / moments on and off, plus the
# residual read from one cached row (row stride 0: what the epilogue costs without the residual's
# memory latency).
cd "$(dirname "$0")/.."
if [ $# -eq 0 ]; then
  set -- "8 768 1 1 1 128 128 128" "8 768 1 1 0 128 128 128" "8 768 1 0 1 128 128 128" \
         "8 768 1 0 0 128 128 128" "8 768 1 1 1 128 128 0"
fi
for v in "$@"; do
  timeout -k 10 60 ./tools/conv_stamp $v || exit $?
done
