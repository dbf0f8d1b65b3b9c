# round 6 session c: PMC traffic passes (with launch sequence) + clock / MFMA-busy pass of one fast step
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u tools/decode_stream_ab.py > gpurun_out/r06c_decode_stream_ab.log 2>&1; rc=$?; echo "decode stream exit $rc"
case $rc in 124|134|137|139) exit $rc;; esac
OUT=gpurun_out/r06c_pmc bash tools/pmc_bench.sh > gpurun_out/r06c_pmc.log 2>&1 || exit $?
rm -rf gpurun_out/r06c_clk
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv \
  -d gpurun_out/r06c_clk -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-validate \
  > gpurun_out/r06c_clk.log 2>&1 || exit $?
python tools/pmc_clock.py gpurun_out/r06c_clk > gpurun_out/r06c_pmc_clock.txt
python tools/traffic_split.py --fetch gpurun_out/r06c_pmc/FETCH_SIZE --write gpurun_out/r06c_pmc/WRITE_SIZE \
  > gpurun_out/r06c_split_gemm.txt 2>&1
python tools/traffic_split.py --fetch gpurun_out/r06c_pmc/FETCH_SIZE --write gpurun_out/r06c_pmc/WRITE_SIZE \
  --family attention_fwd > gpurun_out/r06c_split_attn.txt 2>&1
python tools/bench_traffic.py --fetch gpurun_out/r06c_pmc/FETCH_SIZE --write gpurun_out/r06c_pmc/WRITE_SIZE \
  --preset fast --source "profiles/r06c_pmc_bench_fast.txt (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one fast step, round 6)" \
  --summary gpurun_out/r06c_pmc_summary.txt --out gpurun_out/r06c_bench_traffic.json > gpurun_out/r06c_traffic.log 2>&1
# raw per-dispatch CSVs are large: keep only what the summaries need
find gpurun_out/r06c_pmc gpurun_out/r06c_clk -name '*.csv' -size +20M -delete
echo done1
# halo L2 prefetch (RDMI_HALO_PREF, opt-in): bits and interleaved kernel A/B
timeout -k 10 300 python -u tools/conv_bits.py > gpurun_out/r06c_convbits_0.txt 2>&1 || exit $?
RDMI_HALO_PREF=1 timeout -k 10 300 python -u tools/conv_bits.py > gpurun_out/r06c_convbits_1.txt 2>&1 || exit $?
diff gpurun_out/r06c_convbits_0.txt gpurun_out/r06c_convbits_1.txt > /dev/null && echo "halo pref bits: equal" || echo "halo pref bits: DIFFER"
timeout -k 10 600 python -u tools/env_ab.py --var RDMI_HALO_PREF --values 0,1 --bench conv --rounds 2 > gpurun_out/r06c_halo_pref_conv_ab.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/env_ab.py --var RDMI_HALO_PREF --values 0,1 --bench gnconv --rounds 2 > gpurun_out/r06c_halo_pref_gnconv_ab.log 2>&1 || exit $?
echo done2
timeout -k 10 600 python -u tools/gemm_k32_ab.py > gpurun_out/r06c_gemm_k32_ab.log 2>&1; echo "k32 exit $?"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_pipeline_gpu.py -k "k32 or prefetch or decode_stream" > gpurun_out/r06c_new_tests.log 2>&1; echo "new tests exit $?"
