mkdir -p gpurun_out
run() { timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_tmp.log 2>&1 || return 1; grep metric gpurun_out/ab_tmp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['per_kernel']['attention_fwd']['tflops'], d['roofline']['per_kernel']['implicit_gemm']['tflops'])"; }
export RDMI_VAE_ELEM_CAP=999999999999
timeout -k 10 300 python -u tools/vae_batch_probe.py || exit 1
echo "VB16"; run --vae-batch 16 || exit 1
echo "VB75"; run --vae-batch 75 || exit 1
echo "VB38"; run --vae-batch 38 || exit 1
echo "VB16"; run --vae-batch 16 || exit 1
