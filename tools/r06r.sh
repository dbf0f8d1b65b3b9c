# round 6 session q: n-tile-per-XCD order for the two-workgroups-per-CU halo conv (RDMI_CONV_NXCD=1) against
# the default grouped order (8): each XCD's L2 then holds one n-tile's weights.  Bitwise check per shape.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u tools/conv_ab.py --env RDMI_CONV_NXCD --values 0,1 --rounds 4 --only "512" \
  > gpurun_out/r06r_nxcd_ab.log 2>&1; rc=$?; echo "ab1 exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u tools/conv_ab.py --env RDMI_CONV_NXCD --values 0,1 --rounds 4 --only "256" \
  >> gpurun_out/r06r_nxcd_ab.log 2>&1; echo "ab2 exit $?"
timeout -k 10 500 python -u tools/pipe_env_ab.py --var RDMI_CONV_NXCD --values 0,1 --rounds 3 --steps 1 \
  > gpurun_out/r06r_nxcd_pipe_ab.log 2>&1; echo "pipe exit $?"
