# Engine choice re-measured after the K-loop VALU cuts: the two-workgroups-per-CU halo conv for every
# Cout % 128 == 0 conv (RDMI_CONV_HALO=3) vs the default (256-wide ping-pong for Cout % 256 == 0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 10 200 python -u tools/kbench.py --only conv,gnconv --iters 20 | sed 's/^/dflt /' && RDMI_CONV_HALO=3 timeout -k 10 200 python -u tools/kbench.py --only conv,gnconv --iters 20 | sed 's/^/occ2 /' ) > gpurun_out/r03x_kbench.log 2>&1 || exit $?
for r in 1 2; do
  for m in 2 3; do
    RDMI_CONV_HALO=$m bash tools/hb.sh timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-validate > gpurun_out/r03x_halo${m}_$r.log 2>&1 || exit $?
    echo "halo=$m run $r: $(tail -1 gpurun_out/r03x_halo${m}_$r.log | cut -c1-160)" >> gpurun_out/r03x_halo_ab.log
  done
done
