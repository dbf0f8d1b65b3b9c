# round 6 session l: segment breakdown (in-kernel stamps) of the two-workgroups-per-CU halo conv on the
# pipeline's default GroupNorm path (in_affine table) at its heaviest shapes, against the plain conv
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
run() { timeout -k 10 60 ./tools/conv_stamp "$@" >> gpurun_out/r06l_conv_stamp.log 2>&1; }
rm -f gpurun_out/r06l_conv_stamp.log
run 8 768 1 1 1 128 128 128 1 && run 8 768 1 0 0 128 128 128 1 && run 8 768 1 0 1 128 128 128 1 && \
run 8 768 0 0 0 128 128 128 0 && run 8 768 0 1 1 128 128 128 0 && \
run 8 384 1 1 1 256 256 256 1 && run 8 384 1 0 0 256 256 256 1 && \
run 4 768 1 0 1 256 128 128 1 && echo "stamps ok"
