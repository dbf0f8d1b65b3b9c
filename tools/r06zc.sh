# round 6 session q: RDMI_XFORM_PRIO in the pipeline (interleaved, bitwise check)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u tools/pipe_env_ab.py --var RDMI_XFORM_PRIO --values 0,1 --rounds 5 --steps 1 \
  > gpurun_out/r06zc_xprio_pipe_ab.log 2>&1; echo "pipe exit $?"
