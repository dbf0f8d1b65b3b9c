set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or groupnorm" > gpurun_out/abl_tests.log 2>&1
for h in 0 2; do echo "== HALO=$h" >> gpurun_out/abl.log; RDMI_CONV_HALO=$h timeout -k 5 100 python tools/kbench.py --only conv >> gpurun_out/abl.log 2>&1; done
