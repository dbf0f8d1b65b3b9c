# round 6 session q: the GroupNorm halo transform at s_setprio 2 (RDMI_XFORM_PRIO=1) in the two-workgroups-per-CU conv
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u tools/conv_ab.py --env RDMI_XFORM_PRIO --values 0,1 --rounds 4 --only "gn" \
  > gpurun_out/r06zb_xprio_ab.log 2>&1; echo "ab exit $?"
timeout -k 10 300 python -u tools/conv_ab.py --env RDMI_XFORM_PRIO --values 0,1 --rounds 4 --only "full" \
  >> gpurun_out/r06zb_xprio_ab.log 2>&1; echo "ab2 exit $?"
