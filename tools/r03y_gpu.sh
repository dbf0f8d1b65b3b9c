# Default halo engine -> two workgroups per CU for every Cout % 128 == 0 conv: output bits vs the 256-wide
# form (RDMI_CONV_HALO=2), full GPU test suite, smoke, bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/conv_bits.py > gpurun_out/r03y_bits_new.txt 2>&1 || exit $?
RDMI_CONV_HALO=2 timeout -k 10 200 python -u tools/conv_bits.py > gpurun_out/r03y_bits_old.txt 2>&1 || exit $?
( diff gpurun_out/r03y_bits_old.txt gpurun_out/r03y_bits_new.txt && echo "BITWISE EQUAL" ) > gpurun_out/r03y_bits_diff.txt 2>&1 || true
bash tools/hb.sh timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread > gpurun_out/r03y_gpu_tests.log 2>&1; rc=$?
echo "tests exit $rc"
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/hb.sh timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.log 2>&1 || exit $?
bash tools/hb.sh timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r03y_bench.log 2>&1 || exit $?
