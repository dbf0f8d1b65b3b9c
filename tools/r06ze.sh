# round 6 session q: the halo conv's epilogue at s_setprio 2 (RDMI_EPI_PRIO=1): per shape, then in the pipeline
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u tools/conv_ab.py --env RDMI_EPI_PRIO --values 0,1 --rounds 3 > gpurun_out/r06ze_eprio_ab.log 2>&1
rc=$?; echo "ab exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 700 python -u tools/pipe_env_ab.py --var RDMI_EPI_PRIO --values 0,1 --rounds 4 --steps 1 \
  > gpurun_out/r06ze_eprio_pipe_ab.log 2>&1; echo "pipe exit $?"
