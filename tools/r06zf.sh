# round 6 session q: GPU tests + smoke of the committed final tree (epilogue-priority switch added, off by default)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash tools/hb.sh timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 \
  --timeout-method thread > gpurun_out/r06zf_gpu_tests.log 2>&1; rc=$?; echo "tests exit $rc"; fatal $rc && exit $rc
bash tools/hb.sh timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zf_smoke.log 2>&1
echo "smoke exit $?"
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r06zf_bench.log 2>&1; echo "bench exit $?"
