cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
B=rollingdepth_amd/_lib/librdmi_base.so; N=rollingdepth_amd/_lib/librdmi.so
RDMI_LIB=$N timeout -k 10 300 python -u tools/attn_bits.py --pipe > gpurun_out/r06a_bits_new.txt 2>&1 || exit $?
RDMI_LIB=$B timeout -k 10 300 python -u tools/attn_bits.py --pipe > gpurun_out/r06a_bits_base.txt 2>&1 || exit $?
diff gpurun_out/r06a_bits_base.txt gpurun_out/r06a_bits_new.txt && echo BITS_EQUAL
for r in 1 2; do for v in base new; do lib=$B; [ $v = new ] && lib=$N; echo "== round $r $v"
RDMI_LIB=$lib timeout -k 10 300 python -u tools/kbench.py --only attn,attn512 --iters 8 || exit $?
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_aligner_gpu.py tests/test_kernels_gpu.py -k "merge or fused_input_groupnorm or attention or attn" > gpurun_out/r06a_gpu_tests.log 2>&1; echo "tests exit $?"
