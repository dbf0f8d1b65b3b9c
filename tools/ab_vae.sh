mkdir -p gpurun_out
run() { timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_tmp.log 2>&1 || return 1; grep metric gpurun_out/ab_tmp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['per_kernel']['attention_fwd']['tflops'], d['roofline']['per_kernel']['implicit_gemm']['tflops'])"; }
echo "VB75"; run || exit 1
echo "VB75 empty_cache"; RDMI_PROBE_EMPTY_CACHE=1 run || exit 1
echo "VB16 empty_cache"; RDMI_PROBE_EMPTY_CACHE=1 run --vae-batch 16 || exit 1
