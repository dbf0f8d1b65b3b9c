# round 6 session e: tile-group sweep of the plain halo convs (fabric traffic 2.1x), bench-level A/B of
# the halo L2 prefetch (RDMI_HALO_PREF) on the fast preset, interleaved
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/env_ab.py --var RDMI_GEMM_GROUP --values 8,2,32,128 --bench conv --rounds 2 \
  > gpurun_out/r06e_group_conv_ab.log 2>&1 || exit $?
for r in 1 2; do for v in 0 1; do
  RDMI_HALO_PREF=$v timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-validate \
    > gpurun_out/r06e_bench_pref${v}_r$r.log 2>&1 || exit $?
  echo "pref=$v round $r: $(grep -o '"value": [0-9.]*' gpurun_out/r06e_bench_pref${v}_r$r.log)"
done; done
