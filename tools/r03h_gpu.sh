# Round-3 session-2 GPU batch: aligner tests + timing, attention stamps, fast1024 / full preset benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/hb.sh timeout -k 10 300 python -u -m pytest tests/test_aligner_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03h_aligner_tests.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 200 python -u tools/kbench.py --only aligner --iters 30 > gpurun_out/r03h_kbench_aligner.log 2>&1 || exit $?
timeout -k 10 120 ./tools/attn_stamp 8 27648 > gpurun_out/r03h_attn_stamp.log 2>&1 || exit $?
timeout -k 10 120 ./tools/attn_stamp 25 6912 >> gpurun_out/r03h_attn_stamp.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u bench.py --preset fast1024 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03h_bench_fast1024.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 500 python -u bench.py --preset full --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03h_bench_full.log 2>&1 || exit $?
