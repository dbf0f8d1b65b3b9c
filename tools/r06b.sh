# round 6 session b: f16 error budget per stage, shared-GPU rehearsal of the multi-rank bench line
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
RDMI_BENCH_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --frames-total 30 --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/r06b_shared2.log 2>&1; rc=$?; echo "shared2 exit $rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u tools/error_budget.py sd2_768 sd2_1024 > gpurun_out/r06b_error_budget.log 2>&1; echo "budget exit $?"
