set -e
mkdir -p gpurun_out
for v in 0 1 2 3; do RDMI_ATTN_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" >> gpurun_out/abl_tests.log 2>&1; done
for r in 1 2; do for v in 0 1 2 3; do echo "== VAR=$v" >> gpurun_out/abl.log; RDMI_ATTN_VAR=$v timeout -k 5 100 python tools/kbench.py --only attn >> gpurun_out/abl.log 2>&1; done; done
