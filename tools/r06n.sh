# round 6 session n: fused vs unfused GroupNorm input at the pipeline's batch sizes for the convs the default
# policy leaves unfused (tools/gn_fuse_probe.py)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/gn_fuse_probe.py --rounds 3 > gpurun_out/r06n_gn_fuse_probe.log 2>&1; echo "probe exit $?"
