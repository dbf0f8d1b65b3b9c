set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_processor_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or processor" > gpurun_out/abl_tests.log 2>&1
timeout -k 5 100 python tools/kbench.py --only attn >> gpurun_out/abl.log 2>&1
