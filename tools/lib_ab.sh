#!/bin/bash
# A/B of two builds of librdmi.so on one box: bit fingerprints (tools/conv_bits.py, must be equal for
# bitwise-neutral changes) and interleaved kernel timings (tools/kbench.py).
#   BASE=rollingdepth_amd/_lib/librdmi_base.so OUT=gpurun_out/x KB="--only conv,gnconv" bash tools/lib_ab.sh
cd "$(dirname "$0")/.."
BASE=${BASE:-rollingdepth_amd/_lib/librdmi_base.so}
NEW=${NEW:-rollingdepth_amd/_lib/librdmi.so}
OUT=${OUT:-gpurun_out/lib_ab}
KB=${KB:---only conv,gnconv}
ROUNDS=${ROUNDS:-2}
RDMI_LIB=$NEW timeout -k 10 300 python -u tools/conv_bits.py > ${OUT}_bits_new.txt 2>&1 || exit $?
RDMI_LIB=$BASE timeout -k 10 300 python -u tools/conv_bits.py > ${OUT}_bits_base.txt 2>&1 || exit $?
if diff ${OUT}_bits_base.txt ${OUT}_bits_new.txt > ${OUT}_bits_diff.txt; then echo "bits: equal"; else echo "bits: DIFFER"; fi
for r in $(seq 1 $ROUNDS); do
  for v in base new; do
    lib=$BASE; [ $v = new ] && lib=$NEW
    echo "== round $r $v ($lib)"
    RDMI_LIB=$lib timeout -k 10 300 python -u tools/kbench.py $KB || exit $?
  done
done
