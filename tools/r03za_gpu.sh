# Tile-group size A/B on the final build (RDMI_GEMM_GROUP: m-tiles per group in the XCD-local tile order).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for gsz in 8 4 16; do
    RDMI_GEMM_GROUP=$gsz bash tools/hb.sh timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-validate > gpurun_out/r03za_g${gsz}_$r.log 2>&1 || exit $?
    echo "group=$gsz run $r: $(tail -1 gpurun_out/r03za_g${gsz}_$r.log | cut -c1-160)" >> gpurun_out/r03za_group_ab.log
  done
done
