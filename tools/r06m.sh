# round 6 session m: halo GroupNorm transform with each piece's LDS read issued one piece ahead — bits
# against the previous build, interleaved fused-conv timings, the fused-GroupNorm conv GPU tests
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/r06m_xform_ab KB="--only gnconv" ROUNDS=3 bash tools/lib_ab.sh > gpurun_out/r06m_xform_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "groupnorm or gn" > gpurun_out/r06m_tests.log 2>&1; echo "tests exit $?"
