# Bench A/B on one box: GroupNorm never fused (RDMI_GN_FUSE=0) vs the default policy (Cin <= 256).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for m in 1 0; do
    RDMI_GN_FUSE=$m bash tools/hb.sh timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-validate > gpurun_out/r03v_fuse${m}_$r.log 2>&1 || exit $?
    echo "fuse=$m run $r: $(tail -1 gpurun_out/r03v_fuse${m}_$r.log | cut -c1-160)" >> gpurun_out/r03v_gnfuse_ab.log
  done
done
