#!/bin/bash
# Vector-issue-port occupancy of a kernel from SQ instruction counts (round 5):
# two rocprofv3 --pmc passes per target (tools/traffic_probe.py), each under its own kill timeout,
# summarised by tools/issue_summary.py.  Targets: attention (attn_fwd_d64, and attn_fwd_d64_pipe with
# RDMI_ATTN_PIPE=1) and, for comparison, the 768² GroupNorm-input conv and the plain conv.
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/issue_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F16 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
run() {  # name env args
  local name=$1 envs=$2 args=$3
  for pass in 1 2; do
    eval "P=\$P$pass"
    env $envs timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/${name}_$pass -o run -- \
      python3 tools/traffic_probe.py $args > $OUT/${name}_$pass.log 2>&1
    echo "${name}_$pass ok"
  done
}
run attn "RDMI_ATTN_PIPE=0" "--what attn"
run attn_pipe "RDMI_ATTN_PIPE=1" "--what attn"
run conv_gn "RDMI_CONV_H32=0" "--what conv --variant gn"
run conv_plain "RDMI_CONV_H32=0" "--what conv --variant plain"
