# round 6 session b: windowed-merge test fix, f32 attention XCD A/B, shared-GPU rehearsal of the
# multi-rank bench line, f16 error budget per stage
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
B=rollingdepth_amd/_lib/librdmi_base.so; N=rollingdepth_amd/_lib/librdmi.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_aligner_gpu.py \
  tests/test_kernels_gpu.py -k "merge or fused_input_groupnorm or attention or attn" > gpurun_out/r06b_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
RDMI_LIB=$N timeout -k 10 300 python -u tools/attn_bits.py > gpurun_out/r06b_bits_new.txt 2>&1 || exit $?
for r in 1 2; do for v in base new; do lib=$B; [ $v = new ] && lib=$N; echo "== round $r $v"
RDMI_LIB=$lib timeout -k 10 300 python -u tools/f32_attn_probe.py || exit $?
done; done > gpurun_out/r06b_f32_attn_ab.log 2>&1
RDMI_BENCH_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --frames-total 30 --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/r06b_shared2.log 2>&1; rc=$?; echo "shared2 exit $rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u tools/error_budget.py sd2_768 sd2_1024 > gpurun_out/r06b_error_budget.log 2>&1; echo "budget exit $?"
