# round 6 session q: where the persistent aligner's iteration goes (s_memtime segment sums of workgroups 0 and N-1)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
RDMI_ALIGNER_STAMPS=1 timeout -k 10 200 python -u tools/aligner_ab.py --rounds 1 --values 2 > gpurun_out/r06t_aligner_stamps.log 2>&1
echo "stamps exit $?"
