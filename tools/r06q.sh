# round 6 session q: "one GroupNorm transform per 256 outputs" — the 256-wide 8-wave halo engine (conv_halo_kernel,
# next channel block normalised in the MFMA stream, RDMI_CONV_HALO=2) against the two-workgroups-per-CU engine (=3),
# both with the LDS scale/shift table (RDMI_GN_AFF=0, Cin <= 256), and the default (in_affine table) for reference.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
RDMI_GN_AFF=0 timeout -k 10 300 python -u tools/conv_ab.py --env RDMI_CONV_HALO --values 3,2 --rounds 4 --only "256 384" \
  > gpurun_out/r06q_gn256_engine_ab.log 2>&1; rc=$?; echo "ab1 exit $rc"; fatal $rc && exit $rc
timeout -k 10 300 python -u tools/conv_ab.py --env RDMI_GN_AFF --values 1,0 --rounds 4 --only "256 384" \
  >> gpurun_out/r06q_gn256_engine_ab.log 2>&1; echo "ab2 exit $?"
