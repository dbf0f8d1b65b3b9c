# 256-wide halo conv segment stamps (384² 256->256, 192² 512->512; GroupNorm input + residual + moments and plain).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 10 60 ./tools/conv_stamp 8 384 1 1 1 256 256 && timeout -k 10 60 ./tools/conv_stamp 8 384 0 0 0 256 256 && timeout -k 10 60 ./tools/conv_stamp 8 192 0 0 0 512 512 && timeout -k 10 60 ./tools/conv_stamp 8 96 0 0 0 512 512 ) > gpurun_out/r03r_conv_stamp.log 2>&1 || exit $?
