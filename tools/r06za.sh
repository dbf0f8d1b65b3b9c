# round 6 session q: the session's final library against the session-start build (bcbe0f8) on one box:
# conv bit fingerprints, kernel timings, and interleaved bench lines (is today's 23.05-23.09 the boxes or the code?)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
BASE=rollingdepth_amd/_lib/librdmi_base.so OUT=gpurun_out/r06za KB="--only gnconv,attn" ROUNDS=2 \
  timeout -k 10 700 bash tools/lib_ab.sh > gpurun_out/r06za_lib_ab.log 2>&1; rc=$?; echo "lib_ab exit $rc"
case $rc in 124|134|137|139) exit $rc;; esac
for r in 1 2; do
  for v in base new; do
    lib=rollingdepth_amd/_lib/librdmi.so; [ $v = base ] && lib=rollingdepth_amd/_lib/librdmi_base.so
    RDMI_LIB=$lib timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-validate \
      > gpurun_out/r06za_bench_${v}_$r.log 2>&1; rc=$?; echo "bench $v $r exit $rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
