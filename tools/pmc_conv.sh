#!/bin/bash
# Where the halo convs' wave cycles go: two SQ counter passes per conv variant (tools/traffic_probe.py
# --what conv), each rocprofv3 run under its own kill timeout; stops at the first failing pass.
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_conv}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name probe-args -- counters
  local name=$1; shift
  local args=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python3 tools/traffic_probe.py --what conv $args > $OUT/$name.log 2>&1
  echo "$name ok"
}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
for v in plain gn full; do
  run c128_${v}_1 "--variant $v" $P1
  run c128_${v}_2 "--variant $v" $P2
done
run c256_full_1 "--variant full --res 384 --cin 256" $P1
run c256_full_2 "--variant full --res 384 --cin 256" $P2
run c512_plain_1 "--variant plain --res 192 --cin 512" $P1
run c512_plain_2 "--variant plain --res 192 --cin 512" $P2
