#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own kill timeout) over the
# traffic_probe targets: FETCH/WRITE calibration on a known-bytes copy, HBM traffic of the dominant
# conv, and MFMA/VALU/LDS activity of the level-0 attention.  Stops at the first failing pass.
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_r02}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name what counters...
  local name=$1 what=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python3 tools/traffic_probe.py --what $what > $OUT/$name.log 2>&1
  echo "$name ok"
}
run copy_fetch copy FETCH_SIZE
run copy_write copy WRITE_SIZE
run conv_fetch conv FETCH_SIZE
run conv_write conv WRITE_SIZE
run conv_sq conv SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT
run attn_sq1 attn SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run attn_sq2 attn SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT
run attn_fetch attn FETCH_SIZE
