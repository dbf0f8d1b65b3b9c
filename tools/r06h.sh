# round 6 session h: 4-rank rehearsal of the multi-rank bench path (all ranks on the one GPU, gloo),
# with the per-rank phase / collective fields
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
RDMI_BENCH_SHARED_GPU=1 bash tools/hb.sh timeout -k 10 600 python -u bench.py --gpus 4 --frames-total 30 --steps 2 \
  --warmup 1 --no-cpu-baseline > gpurun_out/r06h_shared4.log 2>&1; echo "shared4 exit $?"
