# round 6 session q: one more default bench line of the final tree on whatever box this call lands on
# (the box-to-box spread of one build)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06z_bench_$1.log 2>&1; echo "bench exit $?"
