# Paper preset N=1 anchor on the build with the one-tile-ahead f32x3 attention.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/hb.sh timeout -k 10 750 python -u bench.py --preset paper --frames-total 500 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03m_bench_paper500.log 2>&1 || exit $?
