# occ2 conv K-loop addressing (four swizzled A offsets per K-tile, DMA K-step in soffset): A/B by stamps
# (output bits must match), conv parity tests, fast-preset bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( for v in "1 1 1" "1 0 0" "0 0 0"; do timeout -k 10 60 ./tools/conv_stamp_old 8 768 $v && timeout -k 10 60 ./tools/conv_stamp 8 768 $v || exit 1; done ) > gpurun_out/r03o_conv_ab.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "conv" > gpurun_out/r03o_conv_tests.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03o_bench.log 2>&1 || exit $?
