# round 6 session o: GroupNorm fusion policy in the pipeline — old rule (Cin <= 256, RDMI_GN_FUSE=3) against
# the new default (also Cout <= 384), fast preset forward interleaved in one process, then the GN GPU tests
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/hb.sh timeout -k 10 900 python -u tools/pipe_env_ab.py --var RDMI_GN_FUSE --values 3,1 --rounds 4 --steps 2 \
  > gpurun_out/r06o_gn_fuse_pipe_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "groupnorm or gn" > gpurun_out/r06o_tests.log 2>&1; echo "tests exit $?"
