#!/bin/bash
# SQ counter passes of the 128-channel 768² conv under both settings of a build switch
# (default RDMI_CONV_H32: the 32×32×16 halo conv vs the two-workgroups-per-CU 16×16×32 one).
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_conv_ab}
ENVV=${ENVV:-RDMI_CONV_H32}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
for v in 0 1; do
  for var in ${VARS:-plain full}; do
    for pass in 1 2; do
      eval "P=\$P$pass"
      export $ENVV=$v; timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/${var}_${v}_$pass -o run -- \
        python3 tools/traffic_probe.py --what conv --variant $var > $OUT/${var}_${v}_$pass.log 2>&1
      echo "${var}_${v}_$pass ok"
    done
  done
done
