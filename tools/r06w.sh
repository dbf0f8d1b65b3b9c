# round 6 session q: aligner tests after the workspace change (persistent region only in opt-in mode 2), smoke
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_aligner_gpu.py tests/test_pipeline_gpu.py \
  > gpurun_out/r06w_aligner_pipeline_tests.log 2>&1; rc=$?; echo "tests exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06w_smoke.log 2>&1; echo "smoke exit $?"
