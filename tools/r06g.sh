# round 6 session g: fast1024 (configs[2]) and full (configs[3]) bench lines on the final build
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/hb.sh timeout -k 10 500 python -u bench.py --preset fast1024 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r06g_bench_fast1024.log 2>&1; rc=$?; echo "fast1024 exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
bash tools/hb.sh timeout -k 10 600 python -u bench.py --preset full --steps 1 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r06g_bench_full.log 2>&1; echo "full exit $?"
