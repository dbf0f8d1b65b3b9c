# round 6 session q: the persistent single-launch aligner (aligner_persist_k) — bitwise tests against the
# two- and three-launch loops, then the fast-preset A/B and a pipeline bench line.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_aligner_gpu.py \
  > gpurun_out/r06s_aligner_tests.log 2>&1; rc=$?; echo "tests exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u tools/aligner_ab.py --rounds 3 --values 1,2,0 > gpurun_out/r06s_aligner_ab.log 2>&1
rc=$?; echo "ab exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u tools/pipe_env_ab.py --var RDMI_ALIGNER_FUSED --values 1,2 --rounds 3 --steps 1 \
  > gpurun_out/r06s_aligner_pipe_ab.log 2>&1; echo "pipe exit $?"
