# round 6 session d2: paper preset (configs[4]) bench at the default precision (heartbeat: long silent steps)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/hb.sh timeout -k 10 1050 python -u bench.py --preset paper --steps 1 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r06d_bench_paper.log 2>&1; echo "paper exit $?"
