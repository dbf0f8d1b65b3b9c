# attn_fwd_d64 DMA addressing (tile step in soffset for whole tiles, SGPR LDS destinations): output bits
# vs the previous library, attention kbench A/B, attention + processor parity tests, bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/conv_bits.py > gpurun_out/r03w_bits_new.txt 2>&1 || exit $?
RDMI_LIB=tools/librdmi_ab_old.so timeout -k 10 200 python -u tools/conv_bits.py > gpurun_out/r03w_bits_old.txt 2>&1 || exit $?
( diff gpurun_out/r03w_bits_old.txt gpurun_out/r03w_bits_new.txt && echo "BITWISE EQUAL" ) > gpurun_out/r03w_bits_diff.txt 2>&1 || true
( for r in 1 2; do RDMI_LIB=tools/librdmi_ab_old.so timeout -k 10 200 python -u tools/kbench.py --only attn --iters 20 | sed 's/^/old /' && timeout -k 10 200 python -u tools/kbench.py --only attn --iters 20 | sed "s/^/new /"; done ) > gpurun_out/r03w_kbench_ab.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_processor_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attention or attn or processor" > gpurun_out/r03w_attn_tests.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03w_bench.log 2>&1 || exit $?
