# f32 engine two-workgroups-per-CU default: f32 parity tests, then the paper preset at 500 frames.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/hb.sh timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py tests/test_processor_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03k_f32_tests.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 750 python -u bench.py --preset paper --frames-total 500 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03k_bench_paper500.log 2>&1 || exit $?
