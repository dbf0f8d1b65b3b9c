# round 6 session q: persistent aligner with two workgroups per frame (gradient rounds split) — bitwise tests,
# A/B against the two-launch loop, stamps
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_aligner_gpu.py -k "fused_loop" \
  > gpurun_out/r06x_aligner_tests.log 2>&1; rc=$?; echo "tests exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u tools/aligner_ab.py --rounds 3 --values 1,2 > gpurun_out/r06x_aligner_ab.log 2>&1
rc=$?; echo "ab exit $rc"; fatal $rc && exit $rc
RDMI_ALIGNER_STAMPS=1 timeout -k 10 200 python -u tools/aligner_ab.py --rounds 1 --values 2 > gpurun_out/r06x_aligner_stamps.log 2>&1
echo "stamps exit $?"
