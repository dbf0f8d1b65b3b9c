mkdir -p gpurun_out
run() { timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_tmp.log 2>&1 || return 1; grep metric gpurun_out/ab_tmp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['per_kernel']['attention_fwd']['tflops'], d['roofline']['per_kernel']['implicit_gemm']['tflops'])"; }
echo "default"; run || exit 1
echo "CONV_HALO=3"; RDMI_CONV_HALO=3 run || exit 1
echo "default"; run || exit 1
echo "CONV_HALO=3"; RDMI_CONV_HALO=3 run || exit 1
