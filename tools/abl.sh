set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or groupnorm or attention" > gpurun_out/abl_tests.log 2>&1
RDMI_CONV_HALO=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or groupnorm" >> gpurun_out/abl_tests.log 2>&1
for r in 1 2; do for h in 0 1 2; do echo "== HALO=$h" >> gpurun_out/abl.log; RDMI_CONV_HALO=$h timeout -k 5 100 python tools/kbench.py --only conv >> gpurun_out/abl.log 2>&1; done; done
timeout -k 5 100 python tools/kbench.py --only attn >> gpurun_out/abl.log 2>&1
