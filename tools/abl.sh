set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or gemm" > gpurun_out/abl_tests.log 2>&1
for g in 1 8; do for d in 0 1 8; do RDMI_GEMM_GROUP=$g RDMI_GEMM_DBG=$d timeout -k 5 60 python tools/gemm_ablate.py >> gpurun_out/abl.log 2>&1; done; done
RDMI_GEMM_PP=2 RDMI_GEMM_GROUP=8 timeout -k 5 100 python tools/kbench.py --only conv,gemm >> gpurun_out/abl.log 2>&1
