# round 6 session q: the attention softmax block at s_setprio 2 (RDMI_ATTN_SPRIO=1) against the default
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/attn_env_ab.py --env RDMI_ATTN_SPRIO --values 0,1 --rounds 4 > gpurun_out/r06zd_sprio_ab.log 2>&1
echo "ab exit $?"
