# round 6 session i: the 32x32x16 halo conv with its GroupNorm transform inlined (no scratch) against the
# default two-workgroups-per-CU engine: bits + interleaved per-shape timing, then the h32 GPU tests
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/conv_ab.py --env RDMI_CONV_H32 --values 0,1 --rounds 3 > gpurun_out/r06i_h32_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "h32 or fused_input_groupnorm" > gpurun_out/r06i_h32_tests.log 2>&1; echo "tests exit $?"
