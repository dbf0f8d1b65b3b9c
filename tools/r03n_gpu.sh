# occ2 conv segment stamps (768² 128→128): full epilogue / GN only / plain.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 10 60 ./tools/conv_stamp 8 768 1 1 1 && timeout -k 10 60 ./tools/conv_stamp 8 768 1 0 0 && timeout -k 10 60 ./tools/conv_stamp 8 768 0 0 0 && timeout -k 10 60 ./tools/conv_stamp 8 768 0 1 1 ) > gpurun_out/r03n_conv_stamp.log 2>&1 || exit $?
