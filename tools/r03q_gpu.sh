# Engine-wide DMA addressing (soffset K step, SGPR LDS destinations): output bits vs the previous library,
# kbench conv / gemm A/B, all kernel parity tests, fast-preset bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/conv_bits.py > gpurun_out/r03q_bits_new.txt 2>&1 || exit $?
RDMI_LIB=tools/librdmi_ab_old.so timeout -k 10 200 python -u tools/conv_bits.py > gpurun_out/r03q_bits_old.txt 2>&1 || exit $?
( diff gpurun_out/r03q_bits_old.txt gpurun_out/r03q_bits_new.txt && echo "BITWISE EQUAL" ) > gpurun_out/r03q_bits_diff.txt 2>&1 || true
( RDMI_LIB=tools/librdmi_ab_old.so timeout -k 10 200 python -u tools/kbench.py --only conv,gemm --iters 20 | sed 's/^/old /' && timeout -k 10 200 python -u tools/kbench.py --only conv,gemm --iters 20 | sed "s/^/new /" ) > gpurun_out/r03q_kbench_ab.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread  > gpurun_out/r03q_conv_tests.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03q_bench.log 2>&1 || exit $?
