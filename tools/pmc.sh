# PMC passes over one kernel shape (tools/attn_probe.py); one pass per rocprofv3 run
set -e
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp; cd - > /dev/null
W=${WHAT:-attn}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/attn_probe.py --what $W ${PROBE_ARGS:-} > $OUT/p$i.log 2>&1
done
