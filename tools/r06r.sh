# round 6 session q: n-tile-per-XCD order for the two-workgroups-per-CU halo conv (RDMI_GEMM_GROUP=-1) against
# the default grouped order (8): each XCD's L2 then holds one n-tile's weights.  Bitwise check per shape.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u tools/conv_ab.py --env RDMI_GEMM_GROUP --values 8,-1 --rounds 4 --only "512" \
  > gpurun_out/r06r_nxcd_ab.log 2>&1; rc=$?; echo "ab1 exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u tools/conv_ab.py --env RDMI_GEMM_GROUP --values 8,-1 --rounds 4 --only "256" \
  >> gpurun_out/r06r_nxcd_ab.log 2>&1; echo "ab2 exit $?"
