#!/bin/bash
# Issue-port / MFMA-busy PMC of the f32 path's engines (round 5): the bf16x3 conv at two VAE shapes and
# the x6 / exact Linear, two rocprofv3 --pmc passes each (counter sets of tools/issue_pmc.sh), summarised
# by tools/issue_summary.py.
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/f32_issue_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F16 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
ONLY=${ONLY:-}
run() {  # name env args
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $1 "* ]]; then return 0; fi
  local name=$1 envs=$2 args=$3
  for pass in 1 2; do
    eval "P=\$P$pass"
    env $envs timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/${name}_$pass -o run -- \
      python3 tools/traffic_probe.py $args > $OUT/${name}_$pass.log 2>&1
    echo "${name}_$pass ok"
  done
}
run x3conv_384 "RDMI_F32_X3=1" "--what f32conv --batch 4 --res 384 --cin 256"
run x3conv_768 "RDMI_F32_X3=1" "--what f32conv --batch 2 --res 768 --cin 128"
run x6gemm "RDMI_F32_X3=6" "--what f32gemm --batch 12 --cin 320"
run x6conv_384 "RDMI_F32_X3=6" "--what f32conv --batch 4 --res 384 --cin 256"
run x6attn "RDMI_F32_X3=conv RDMI_F32_X6=1" "--what f32attn --batch 2"
run x3attn "RDMI_F32_X3=1" "--what f32attn --batch 2"
